"""Top kernels of one replayed C2 training step with their PMC counters
(tools/gpu_step_pmc.sh output): launches per step, time per step, MFMA-busy
share, HBM bytes and GB/s per launch.

python tools/step_pmc_report.py gpurun_out/steppmc [top] [--also sub,sub] > profiles/r02/step_top_kernels.md

--also: after the top table, every kernel whose name contains one of the
substrings (e.g. the VALU attention kernels, to place them on the HBM /
latency roofline).

Kernels are keyed by (name, grid size, workgroup size). Time per step comes
from the un-profiled kernel trace (last replayed step); counters are averaged
over every dispatch of the key in the PMC runs. Corrections per
MI355X_MICROARCH.md: HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB; gfx950
FETCH_SIZE counts half of a 16-B/lane streaming read); MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 4 SIMDs * 256 CUs).
"""
import collections
import csv
import glob
import os
import sys

CUS = 256
HBM_PEAK = 8000.0  # GB/s (MI355X_MICROARCH.md)


def short(n):
    n = n.replace("_ZN5fpnmt11gemm_kernelIDF16bLi", "gemm_kernel<bf16,").replace("void fpnmt::", "")
    n = n.replace("_ZN5fpnmt17gemm_small_kernelIDF16bLi", "gemm_small_kernel<bf16,")
    return n.split("EEEvNS_")[0].split("(fpnmt::")[0].split("(long")[0].split("(int")[0][:70]


def step_rows(trace):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "amsgrad_kernel" in r["Kernel_Name"]]
    return rows[idx[-2] + 1: idx[-1] + 1]


def pmc(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            dd = disp[(r["Dispatch_Id"], key)]
            dd[r["Counter_Name"]] = float(r["Counter_Value"])
            dd["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (_, key), cs in disp.items():
            for c, v in cs.items():
                acc[key][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    argv = list(sys.argv[1:])
    also = []
    if "--also" in argv:
        i = argv.index("--also")
        also = [x for x in argv[i + 1].split(",") if x]
        del argv[i:i + 2]
    d = argv[0]
    top = int(argv[1]) if len(argv) > 1 else 5
    step = step_rows(glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))[0])
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) *
               int(r.get("Grid_Size_Z", 1) or 1), int(r["Workgroup_Size_X"]))
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    pm = pmc(d)
    busy = sum(t for _, t in agg.values())
    print(f"# C2 training step: top {top} kernels (one replayed step: {len(step)} kernels, "
          f"{span:.0f} us span, {busy:.0f} us busy)\n")
    print("| kernel | grid / wg | launches | us / step | avg us | MFMA busy | HBM MB / launch | HBM GB/s | HBM frac |")
    print("|---|---|---|---|---|---|---|---|---|")
    ranked = sorted(agg.items(), key=lambda kv: -kv[1][1])
    rows = ranked[:top]
    extra = [kv for kv in ranked[top:] if any(a in kv[0][0] for a in also)]
    for item in rows + ([None] if extra else []) + extra:
        if item is None:
            print("| *(selected kernels below the top rows)* | | | | | | | | |")
            continue
        key, (n, t) = item
        cs = pm.get(key, {})
        gui, mf = cs.get("GRBM_GUI_ACTIVE"), cs.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfma = f"{100 * mf / (gui / 8 * 4 * CUS):.1f} %" if gui and mf is not None else "n/a"
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            byts = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            gbs = f"{byts / (t / n * 1e3):.0f}"
            mb = f"{byts / 1e6:.1f}"
            frac = f"{byts / (t / n * 1e3) / HBM_PEAK:.2f}"
        else:
            gbs = mb = frac = "n/a"
        print(f"| `{short(key[0])}` | {key[1]} / {key[2]} | {n} | {t:.0f} | {t / n:.1f} | {mfma} | {mb} | {gbs} | {frac} |")


if __name__ == "__main__":
    main()
