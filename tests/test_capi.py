"""The C-ABI library loads on a GPU-less host and exports exactly the entry
points include/fpnmt.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "fpnmt.h")).read()
    return sorted(set(re.findall(r"\b(fpnmt_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from fpnmt import _lib as L
    lib = ctypes.CDLL(L.LIB_PATH)
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from fpnmt import _lib as L
    assert sorted(_header_symbols()) == sorted(L.ALL_SYMBOLS)


def test_version_and_error_path():
    from fpnmt import _lib as L
    assert L.lib.fpnmt_version() == 100
    # argument validation happens before any HIP call
    d = L.GemmDesc()
    d.m, d.n, d.k, d.batch, d.batch_inner = 4, 4, 4, 1, 0  # batch_inner 0 is invalid
    rc = L.lib.fpnmt_gemm(d, 1, 1, 1, None, None, None, None)
    assert rc == -1
    assert b"negative size" in L.lib.fpnmt_last_error() or b"gemm" in L.lib.fpnmt_last_error()
    rc = L.lib.fpnmt_gemm(None, None, None, None, None, None, None, None)
    assert rc == -1 and b"null" in L.lib.fpnmt_last_error()


def test_struct_layouts_match_header():
    """ctypes mirrors of the descriptor structs have the C sizes."""
    from fpnmt import _lib as L
    assert ctypes.sizeof(L.ConvDesc) == 16 * 4
    assert ctypes.sizeof(L.AdamDesc) == 10 * 4
    assert ctypes.sizeof(L.AttnDesc) == 6 * 4 + 5 * 8 + 8 + 4 * 8


def test_library_build_id_matches_tree():
    """The in-tree libfpnmt.so was built from exactly the committed csrc/ +
    Makefile + include/fpnmt.h (csrc/Makefile BUILD_ID)."""
    from fpnmt import _lib as L
    assert L.library_build_id() == L.tree_build_id()
    L.assert_in_tree()


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library built from other sources than the tree's fails
    assert_in_tree(), which bench.py, smoke() and the GPU tests call."""
    import shutil
    import pytest
    from fpnmt import _lib as L
    src = tmp_path / "csrc"
    shutil.copytree(L.CSRC_DIR, src)
    hdr = tmp_path / "fpnmt.h"
    shutil.copy(L.HEADER_PATH, hdr)
    assert L.tree_build_id(str(src), str(hdr)) == L.library_build_id()
    with open(src / "common.h", "a") as f:
        f.write("\n// edited after the build\n")
    edited = L.tree_build_id(str(src), str(hdr))
    assert edited != L.library_build_id()
    monkeypatch.setattr(L, "tree_build_id", lambda *a, **k: edited)
    with pytest.raises(RuntimeError, match="built from other sources"):
        L.assert_in_tree()
