"""Per-kernel PMC summary from rocprofv3 --pmc passes (pmc*/pmc_counter_collection.csv).

python tools/pmc_table.py <dir-with-pmcN-subdirs> [--match substr] [--shapes conv_bench_order]

Dispatches are keyed by (kernel name, grid size, workgroup size); values are
averaged over the dispatches of a key. Derived columns (MI355X_MICROARCH.md):
  mfma%   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 4 SIMD * CUs)  — busy share of the matrix pipes
          (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  hbm_MB  (2 * FETCH_SIZE + WRITE_SIZE) KiB -> MB (gfx950 FETCH_SIZE counts half of 16-B/lane streaming reads)
  wait%   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls), idle% SQ_WAIT_ANY / SQ_WAVE_CYCLES
  ldsconf SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import glob
import os
import sys

CUS = 256


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    order = []
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            disp[(r["Dispatch_Id"], key)][r["Counter_Name"]] = float(r["Counter_Value"])
        for (did, key), cs in disp.items():
            if key not in order:
                order.append(key)
            for c, v in cs.items():
                per[key][c].append(v)
    return per, order


def short(name):
    n = name.replace("_ZN5fpnmt11gemm_kernelIDF16bLi", "gemm<").replace("void fpnmt::", "")
    return n.split("EEEvNS_")[0].split("(fpnmt::GemmParams")[0][:58]


def main():
    d = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else None
    per, order = load(d)
    print(f"{'kernel':58s} {'grid':>8s} {'n':>3s} {'mfma%':>6s} {'wait%':>6s} {'idle%':>6s} {'ldsconf':>7s} "
          f"{'hbm_MB':>8s} {'vgpr':>4s}")
    for key in order:
        if match and match not in key[0]:
            continue
        cs = {c: sum(v) / len(v) for c, v in per[key].items()}
        n = max(len(v) for v in per[key].values())
        gui = cs.get("GRBM_GUI_ACTIVE")
        mf = cs.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfma = 100 * mf / (gui / 8 * 4 * CUS) if gui and mf is not None else float("nan")
        wc = cs.get("SQ_WAVE_CYCLES")
        wait = 100 * cs["SQ_WAIT_INST_ANY"] / wc if wc and "SQ_WAIT_INST_ANY" in cs else float("nan")
        idle = 100 * cs["SQ_WAIT_ANY"] / wc if wc and "SQ_WAIT_ANY" in cs else float("nan")
        lc = cs["SQ_LDS_BANK_CONFLICT"] / cs["SQ_LDS_IDX_ACTIVE"] if cs.get("SQ_LDS_IDX_ACTIVE") else float("nan")
        hbm = (2 * cs.get("FETCH_SIZE", float("nan")) + cs.get("WRITE_SIZE", float("nan"))) * 1024 / 1e6
        print(f"{short(key[0]):58s} {key[1]:8d} {n:3d} {mfma:6.1f} {wait:6.1f} {idle:6.1f} {lc:7.3f} {hbm:8.1f}")


if __name__ == "__main__":
    main()
