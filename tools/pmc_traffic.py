"""HBM traffic per launch of the roofline kernel from two separate rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE; kB), with the gfx950 correction
(FETCH_SIZE counts 16-B/lane streaming reads at half size):
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
python tools/pmc_traffic.py fetch.csv write.csv <kernel-substring> <algorithmic bytes> > profiles/roofline_pmc.json"""
import csv
import json
import sys


def per_launch(path, counter, key):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and key in r["Kernel_Name"]]
    return sum(vals) / max(1, len(vals)), len(vals)


fetch, n = per_launch(sys.argv[1], "FETCH_SIZE", sys.argv[3])
write, _ = per_launch(sys.argv[2], "WRITE_SIZE", sys.argv[3])
alg = int(sys.argv[4])
hbm = int((2 * fetch + write) * 1024)
print(json.dumps({
    "kernel": sys.argv[3], "launches": n, "FETCH_SIZE_kB": fetch, "WRITE_SIZE_kB": write,
    "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halves 16B-lane streaming reads)",
    "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg, "reread_factor": round(hbm / alg, 3)}, indent=1))
