"""Top kernels of the R50-FPN headline forward (bench.py --headline-only) with
their MFMA-busy share and HBM fraction, as a markdown table.

python tools/headline_pmc_report.py <kernel_trace.csv of the --stats run> <dir with pmc1..3> [top]

Durations: the kernel trace of the --stats run, keyed by (kernel, grid,
workgroup), averaged per dispatch; counters: tools/pmc_table.py's passes
(SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE, FETCH_SIZE / WRITE_SIZE with the
gfx950 FETCH_SIZE correction). HBM fraction = counted bytes / duration / 8 TB/s.
"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import CUS, load, short  # noqa: E402

HBM_PEAK = 8.0e12


def main():
    trace, pmc_dir = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) *
               int(r.get("Grid_Size_Z", 1) or 1), int(r["Workgroup_Size_X"]))
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    per, _ = load(pmc_dir)
    rows = []
    total = sum(sum(v) for v in dur.values())
    for key, ds in dur.items():
        cs = {c: sum(v) / len(v) for c, v in per.get(key, {}).items()}
        t = sum(ds) / len(ds)
        gui, mf = cs.get("GRBM_GUI_ACTIVE"), cs.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfma = mf / (gui / 8 * 4 * CUS) if gui and mf is not None else float("nan")
        hbm = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs else float("nan")
        rows.append((sum(ds), len(ds), t, key, mfma, hbm))
    rows.sort(key=lambda r: -r[0])
    print(f"Top {top} kernels of the R50-FPN forward at batch 64 (bench.py --headline-only; "
          f"{total * 1e3:.2f} ms of kernel time over the traced passes)\n")
    print("| kernel | grid | launches | avg us | share | MFMA busy | HBM MB / launch | HBM fraction |")
    print("|---|---|---|---|---|---|---|---|")
    for tot, n, t, key, mfma, hbm in rows[:top]:
        frac = hbm / t / HBM_PEAK if hbm == hbm else float("nan")
        print(f"| `{short(key[0])}` | {key[1] // key[2]}x{key[2]} | {n} | {t * 1e6:.1f} | {100 * tot / total:.1f} % | "
              f"{100 * mfma:.1f} % | {hbm / 1e6:.1f} | {frac:.2f} |")


if __name__ == "__main__":
    main()
