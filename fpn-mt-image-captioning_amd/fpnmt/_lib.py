"""ctypes binding of libfpnmt.so (the C-ABI declared in include/fpnmt.h).

The product path has no fallback: if the in-tree library is missing or fails to
load, importing this module raises. Every call is checked and a non-zero
status raises ``RuntimeError(fpnmt_last_error())`` (the reference raises
TF InvalidArgumentError for the same class of shape errors).
"""
from __future__ import annotations

import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# FPNMT_LIBRARY: load another build of the same C-ABI (tools/conv_bench.py
# same-box A/B runs); the default is the in-tree build
IN_TREE_PATH = os.path.join(_HERE, "libfpnmt.so")
LIB_PATH = os.environ.get("FPNMT_LIBRARY") or IN_TREE_PATH


CSRC_DIR = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "fpnmt.h")


def tree_build_id(csrc_dir: str = CSRC_DIR, header: str = HEADER_PATH) -> str:
    """The build id the tree's sources give: sha256 over csrc/*.hip + *.h
    (sorted by name, like make's $(sort)), csrc/Makefile, include/fpnmt.h —
    the digest csrc/Makefile compiles into fpnmt_build_id()."""
    import hashlib
    names = sorted(f for f in os.listdir(csrc_dir) if f.endswith((".hip", ".h")))
    h = hashlib.sha256()
    for p in [os.path.join(csrc_dir, f) for f in names] + [os.path.join(csrc_dir, "Makefile"), header]:
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def library_build_id() -> str:
    return lib.fpnmt_build_id().decode()


def assert_in_tree():
    """bench.py, smoke() and the GPU tests measure the in-tree build only: an
    FPNMT_LIBRARY override pointing elsewhere is an error there, and so is an
    in-tree library built from other sources than the tree's (its compiled-in
    build id differs from the digest of csrc/ + Makefile + include/fpnmt.h)."""
    if os.path.realpath(LIB_PATH) != os.path.realpath(IN_TREE_PATH):
        raise RuntimeError(f"fpnmt: FPNMT_LIBRARY={LIB_PATH} is not the in-tree build {IN_TREE_PATH}; "
                           "unset it for benchmarks, smoke and tests")
    built, tree = library_build_id(), tree_build_id()
    if built != tree:
        raise RuntimeError(f"fpnmt: {LIB_PATH} was built from other sources (build id {built}) than the "
                           f"tree's csrc/ ({tree}); rebuild it with `make -C fpn-mt-image-captioning_amd/csrc`")
    # the library reads no dispatch-tuning variables any more; a stale one in
    # the environment would still mislabel a measurement
    knobs = sorted(k for k in os.environ if k.startswith(("FPNMT_TUNE_", "FPNMT_DBG_")))
    if knobs:
        raise RuntimeError(f"fpnmt: tuning / debug variables set ({', '.join(knobs)}); "
                           "unset them for benchmarks, smoke and tests")

F32, BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_LEAKY, ACT_RELU6 = 0, 1, 2, 3


class GemmDesc(C.Structure):
    _fields_ = [
        ("m", C.c_int), ("n", C.c_int), ("k", C.c_int),
        ("batch", C.c_int), ("batch_inner", C.c_int),
        ("dtype", C.c_int), ("a_trans", C.c_int), ("b_trans", C.c_int),
        ("lda", C.c_longlong), ("ldb", C.c_longlong), ("ldc", C.c_longlong), ("ldr", C.c_longlong),
        ("a_so", C.c_longlong), ("a_si", C.c_longlong), ("b_so", C.c_longlong), ("b_si", C.c_longlong),
        ("c_so", C.c_longlong), ("c_si", C.c_longlong), ("r_so", C.c_longlong), ("r_si", C.c_longlong),
        ("alpha", C.c_float), ("act", C.c_int), ("act_alpha", C.c_float),
        ("accumulate", C.c_int), ("c_f32", C.c_int), ("split_k", C.c_int),
        ("drop_p", C.c_float), ("drop_seed", C.c_ulonglong), ("drop_seed_dev", C.c_void_p),
    ]


class ConvDesc(C.Structure):
    _fields_ = [
        ("n", C.c_int), ("h", C.c_int), ("w", C.c_int), ("c", C.c_int),
        ("k", C.c_int), ("r", C.c_int), ("s", C.c_int),
        ("stride_h", C.c_int), ("stride_w", C.c_int),
        ("pad_t", C.c_int), ("pad_b", C.c_int), ("pad_l", C.c_int), ("pad_r", C.c_int),
        ("dtype", C.c_int), ("act", C.c_int), ("act_alpha", C.c_float),
    ]


class ConvLevel(C.Structure):
    _fields_ = [
        ("n", C.c_int), ("h", C.c_int), ("w", C.c_int),
        ("x", C.c_void_p), ("dz", C.c_void_p), ("residual", C.c_void_p), ("y", C.c_void_p),
    ]


class LnView(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("y", C.c_void_p), ("dy", C.c_void_p), ("mean", C.c_void_p), ("rstd", C.c_void_p),
        ("rows", C.c_longlong), ("pe_rows", C.c_int), ("seed", C.c_ulonglong),
    ]


class AttnDesc(C.Structure):
    _fields_ = [
        ("b", C.c_int), ("h", C.c_int), ("lq", C.c_int), ("lk", C.c_int), ("d", C.c_int),
        ("dtype", C.c_int),
        ("ldq", C.c_longlong), ("ldk", C.c_longlong), ("ldv", C.c_longlong),
        ("ldo", C.c_longlong), ("ldw", C.c_longlong),
        ("scale", C.c_float),
        ("m_sb", C.c_longlong), ("m_sh", C.c_longlong), ("m_si", C.c_longlong), ("m_sj", C.c_longlong),
    ]


class AdamDesc(C.Structure):
    _fields_ = [
        ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("clipnorm", C.c_float),
        ("sched_d_model", C.c_float), ("sched_warmup", C.c_float), ("sched_mult", C.c_float),
        ("sched_warm_pow", C.c_float), ("const_lr", C.c_float), ("grad_scale", C.c_float),
    ]


class WPrepItem(C.Structure):
    _fields_ = [
        ("w_hwio", C.c_void_p), ("scale", C.c_void_p), ("w_ohwi", C.c_void_p), ("w_flip", C.c_void_p),
        ("r", C.c_int), ("s", C.c_int), ("c", C.c_int), ("k", C.c_int),
        ("tile_start", C.c_longlong), ("ld_flip", C.c_longlong),
    ]


class SegPrep(C.Structure):
    _fields_ = [
        ("ohwi", C.c_void_p), ("flip", C.c_void_p), ("scale", C.c_void_p),
        ("r", C.c_int), ("s", C.c_int), ("c", C.c_int), ("k", C.c_int),
        ("ld_flip", C.c_longlong), ("c_magic", C.c_uint32), ("c_shift", C.c_uint32),
    ]


P = C.c_void_p
I = C.c_int
LL = C.c_longlong
F = C.c_float
ULL = C.c_ulonglong
PP = C.POINTER(C.c_void_p)  # a table of device pointers ((C.c_void_p * n)(...))

# name -> argtypes (restype int unless noted); must mirror include/fpnmt.h
SIGNATURES = {
    "fpnmt_version": [],
    "fpnmt_set_workspace": [P, LL],
    "fpnmt_fill_zero": [P, LL, P],
    "fpnmt_fill_zero_grid": [P, LL, I, P],
    "fpnmt_defer_begin": [P, LL],
    "fpnmt_defer_flush": [P],
    "fpnmt_gemm": [C.POINTER(GemmDesc), P, P, P, P, P, P, P],
    "fpnmt_gemm_act_in": [C.POINTER(GemmDesc), P, P, P, P, I, F, P],
    "fpnmt_gemm_wgrad": [C.POINTER(GemmDesc), P, P, P, P],
    "fpnmt_bottleneck_fwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, P],
    "fpnmt_conv2d_fwd": [C.POINTER(ConvDesc), P, P, P, P, P, P, P],
    "fpnmt_conv2d_bwd_data": [C.POINTER(ConvDesc), P, P, P, I, P],
    "fpnmt_conv2d_bwd_data_act": [C.POINTER(ConvDesc), P, P, P, P, I, P],
    "fpnmt_conv2d_bwd_data_mask": [C.POINTER(ConvDesc), P, P, P, I, P, I, P],
    "fpnmt_conv2d_bwd_data_res": [C.POINTER(ConvDesc), P, P, P, P, P],
    "fpnmt_conv2d_bwd_data_res_act": [C.POINTER(ConvDesc), P, P, P, P, P, I, P],
    "fpnmt_conv2d_bwd_filter": [C.POINTER(ConvDesc), P, P, P, P, P],
    "fpnmt_conv2d_bwd_filter_bias": [C.POINTER(ConvDesc), P, P, P, P, P, P],
    "fpnmt_conv2d_fwd_grouped": [C.POINTER(ConvDesc), I, C.POINTER(ConvLevel), P, P, P, P],
    "fpnmt_conv2d_bwd_data_grouped": [C.POINTER(ConvDesc), I, C.POINTER(ConvLevel), P, I, P],
    "fpnmt_conv2d_bwd_data_grouped_act": [C.POINTER(ConvDesc), I, C.POINTER(ConvLevel), P, I, P],
    "fpnmt_conv2d_bwd_data_grouped_mask": [C.POINTER(ConvDesc), I, C.POINTER(ConvLevel), P, I, I, P],
    "fpnmt_conv2d_bwd_filter_grouped": [C.POINTER(ConvDesc), I, C.POINTER(ConvLevel), P, P, P],
    "fpnmt_conv2d_bwd_filter_grouped_bias": [C.POINTER(ConvDesc), I, C.POINTER(ConvLevel), P, P, P, P],
    "fpnmt_weight_prep": [P, I, I, I, I, P, I, P, P, LL, P],
    "fpnmt_weight_prep_batched": [P, I, LL, I, P],
    "fpnmt_act_bwd": [I, LL, I, I, F, P, P, P, P, P, F, ULL, P, P],
    "fpnmt_bias_grad": [I, LL, I, P, P, P],
    "fpnmt_cast": [I, I, LL, P, P, P],
    "fpnmt_dropout": [I, LL, F, ULL, P, P, P, P],
    "fpnmt_add": [I, LL, P, P, P, P],
    "fpnmt_maxpool2d_fwd": [I, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P],
    "fpnmt_maxpool2d_bwd": [I, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P, P],
    "fpnmt_maxpool2d_bwd_act": [I, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, I, F, P, P],
    "fpnmt_fpn_topdown_fwd": [I, I, I, I, I, I, I, I, I, P, P, P, P, P, P],
    "fpnmt_fpn_topdown_bwd": [I, I, I, I, I, I, I, I, I, P, P, P, P, I, P],
    "fpnmt_spatial_softmax_fwd": [I, I, I, I, P, P, P, P, P],
    "fpnmt_spatial_softmax_bwd": [I, I, I, I, P, P, P, P, P, P, P],
    "fpnmt_attention_fwd": [C.POINTER(AttnDesc), P, P, P, P, P, P, P, P],
    "fpnmt_attention_bwd": [C.POINTER(AttnDesc), P, P, P, P, P, P, P, P, P, P],
    "fpnmt_attention_fwd_views": [I, C.POINTER(AttnDesc), PP, PP, PP, PP, PP, PP, PP, P],
    "fpnmt_attention_bwd_views": [I, C.POINTER(AttnDesc), PP, PP, PP, PP, PP, PP, PP, PP, PP, P],
    "fpnmt_view_proj_fwd": [I, I, I, I, I, P, LL, P, P, P, LL, P, LL, F, ULL, P, P],
    "fpnmt_view_proj_bwd_dz": [I, I, I, I, P, LL, P, P, F, ULL, P, P],
    "fpnmt_layernorm_fwd": [I, LL, I, F, P, P, P, P, P, I, P, P, P, P],
    "fpnmt_layernorm_bwd": [I, LL, I, P, P, P, P, P, P, P, P, P, P],
    "fpnmt_layernorm_bwd_drop": [I, LL, I, P, P, P, P, P, P, P, P, P, F, ULL, P, P, P],
    "fpnmt_decoder_targets": [I, I, P, I, LL, P, P, P, P],
    "fpnmt_layernorm_views_fwd": [I, I, I, F, C.POINTER(LnView), P, P, P, F, P, P],
    "fpnmt_layernorm_views_bwd": [I, I, I, C.POINTER(LnView), P, F, P, P, P, P],
    "fpnmt_embed_posenc_fwd": [I, I, I, I, P, P, P, P, P],
    "fpnmt_embed_posenc_bwd": [I, I, I, I, P, P, P, P, P],
    "fpnmt_embed_posenc_fwd_drop": [I, I, I, I, P, P, P, P, F, ULL, P, P],
    "fpnmt_embed_posenc_bwd_drop": [I, I, I, I, P, P, P, P, F, ULL, P, P],
    "fpnmt_xent_fwd_bwd": [I, LL, I, P, LL, P, P, P, LL, F, P],
    "fpnmt_grad_sumsq": [I, P, P, I, P, P, P, F, P, P],
    "fpnmt_amsgrad_step": [C.POINTER(AdamDesc), I, P, P, I, P, P, P, P, P, P, P, P, P, P, P, P],
    "fpnmt_amsgrad_step_prep": [C.POINTER(AdamDesc), I, P, P, I, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "fpnmt_grad_sumsq_part": [I, I, I, P, P, I, P, P, P, F, P, P],
    "fpnmt_amsgrad_step_part": [C.POINTER(AdamDesc), I, I, I, I, P, P, I, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "fpnmt_decode_attention": [I, I, I, I, I, F, P, LL, P, LL, LL, LL, LL, P, I, I, P, LL, P],
    "fpnmt_beam_step": [I, I, I, P, LL, P, P, P, I, I, P, P, I, I, P, P, I, P, P, P],
    "fpnmt_bn_stats": [I, LL, I, P, P, P, P, P, F, P],
    "fpnmt_bn_apply": [I, LL, I, P, P, P, P, P, F, I, P, P, P],
    "fpnmt_bn_bwd": [I, LL, I, P, P, P, P, F, I, P, P, P, P, P, P],
    "fpnmt_bn_stats_sums": [I, LL, I, P, P, P],
    "fpnmt_bn_stats_finalize": [I, P, P, P, P, P, F, P],
    "fpnmt_bn_bwd_sums": [I, LL, I, P, P, P, F, I, P, P, P, P, P, P],
    "fpnmt_bn_bwd_dx": [I, LL, I, P, P, P, P, F, I, P, P, P, P, P],
    "fpnmt_depthwise_fwd": [I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P],
    "fpnmt_depthwise_bwd_data": [I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P],
    "fpnmt_depthwise_bwd_filter": [I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P],
    "fpnmt_image_resize_normalize": [P, I, P, LL, I, I, I, F, F, I, P, P],
}
SIZE_T_FUNCS = {"fpnmt_attention_ws_bytes": [C.POINTER(AttnDesc)]}
LL_FUNCS = {"fpnmt_act_bwd_ws_bytes": [I, LL, I], "fpnmt_defer_peak_bytes": []}
STR_FUNCS = {"fpnmt_last_error": [], "fpnmt_build_id": []}
ALL_SYMBOLS = sorted(list(SIGNATURES) + list(SIZE_T_FUNCS) + list(LL_FUNCS) + list(STR_FUNCS))


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libfpnmt.so not found at {LIB_PATH}; build it with "
            "`make -C fpn-mt-image-captioning_amd/csrc` (or __graft_entry__.build()). "
            "There is no fallback path.")
    lib = C.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    for name, args in SIZE_T_FUNCS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_size_t
    for name, args in LL_FUNCS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_longlong
    for name, args in STR_FUNCS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_char_p
    return lib


lib = _load()


E_ARG, E_UNSUPPORTED, E_HIP = -1, -2, -3  # include/fpnmt.h status codes


def check(status: int, what: str = ""):
    if status != 0:
        msg = lib.fpnmt_last_error().decode(errors="replace")
        raise RuntimeError(f"fpnmt {what} failed ({status}): {msg}")


def call(name: str, *args):
    check(getattr(lib, name)(*args), name)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


WORKSPACE_BYTES = 256 << 20  # split-K partial slabs + ordered-reduction scratch
_ws = {}
_ws_dev = [None]


def _ensure_workspace():
    """Attach the (zeroed) split-K GEMM workspace of the current device."""
    dev = torch.cuda.current_device()
    if _ws_dev[0] == dev:
        return
    buf = _ws.get(dev)
    if buf is None:
        buf = torch.zeros(WORKSPACE_BYTES, dtype=torch.uint8, device=f"cuda:{dev}")
        _ws[dev] = buf
    check(lib.fpnmt_set_workspace(buf.data_ptr(), buf.numel()), "fpnmt_set_workspace")
    _ws_dev[0] = dev


_ws_side = {}


class side_workspace:
    """Attach a second split-K workspace for the calls issued inside (the
    weight-gradient side stream's launches run concurrently with the compute
    stream's, so their partial slabs need memory of their own; kernels bake
    the workspace pointers in at launch)."""

    def __enter__(self):
        _ensure_workspace()
        dev = torch.cuda.current_device()
        buf = _ws_side.get(dev)
        if buf is None:
            buf = torch.zeros(WORKSPACE_BYTES, dtype=torch.uint8, device=f"cuda:{dev}")
            _ws_side[dev] = buf
        check(lib.fpnmt_set_workspace(buf.data_ptr(), buf.numel()), "fpnmt_set_workspace")
        return self

    def __exit__(self, *exc):
        dev = torch.cuda.current_device()
        buf = _ws[dev]
        check(lib.fpnmt_set_workspace(buf.data_ptr(), buf.numel()), "fpnmt_set_workspace")
        return False


DEFER_BYTES = 3 << 30  # deferred-reduction arena (slabs + partials of one backward)
_defer = {}


class deferred_reductions:
    """fpnmt_defer_begin .. fpnmt_defer_flush around a backward: its ordered
    gradient reductions run as a few batched launches at the exit (on the
    then-current stream). The arena is allocated once per device."""

    def __init__(self, enabled=True):
        self.enabled = enabled

    def __enter__(self):
        self.on = False
        if self.enabled and torch.cuda.is_available():
            dev = torch.cuda.current_device()
            buf = _defer.get(dev)
            if buf is None:
                buf = torch.empty(DEFER_BYTES, dtype=torch.uint8, device=f"cuda:{dev}")
                _defer[dev] = buf
            _ensure_workspace()
            check(lib.fpnmt_defer_begin(buf.data_ptr(), buf.numel()), "fpnmt_defer_begin")
            self.on = True
            _defer_active[0] = True
        return self

    def __exit__(self, *exc):
        if self.on:
            _defer_active[0] = False
            check(lib.fpnmt_defer_flush(torch.cuda.current_stream().cuda_stream), "fpnmt_defer_flush")
            # queued bias gradients read their inputs at the flush (enqueued
            # above): the references may go now (stream order protects reuse)
            _defer_keep.clear()
        return False


_defer_active = [False]
_defer_keep = []  # tensors read by queued launches (fpnmt_bias_grad), held until the flush


def defer_checkpoint():
    """Inside deferred_reductions: run the queued reductions now (on the
    current stream) and keep deferring the ones issued after this point, so
    the gradients queued so far are final when this returns (stream order).
    No-op outside a region."""
    if not _defer_active[0]:
        return
    dev = torch.cuda.current_device()
    buf = _defer[dev]
    check(lib.fpnmt_defer_flush(torch.cuda.current_stream().cuda_stream), "fpnmt_defer_flush")
    _defer_keep.clear()
    check(lib.fpnmt_defer_begin(buf.data_ptr(), buf.numel()), "fpnmt_defer_begin")


def defer_keep(t):
    """Hold t until the active deferred region's flush has been enqueued."""
    if _defer_active[0]:
        _defer_keep.append(t)


def defer_active():
    """Inside deferred_reductions (single-stream: the queue's flush reads
    slabs written earlier on the same stream)."""
    return _defer_active[0]


def stream_ptr():
    _ensure_workspace()
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float32:
        return F32
    raise TypeError(f"fpnmt kernels run in float32 or bfloat16, got {dt}")


ACT_CODES = {None: ACT_NONE, "linear": ACT_NONE, "relu": ACT_RELU, "leaky_relu": ACT_LEAKY, "relu6": ACT_RELU6}
