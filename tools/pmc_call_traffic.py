"""HBM bytes per CorrelateFFT call from the rocprofv3 FETCH_SIZE / WRITE_SIZE
passes of tools/gpu_corr_prof.sh (bench.py --workload corr).

Usage: python tools/pmc_call_traffic.py <corrprof_dir> [n] > profiles/corr_pmc_traffic.json

Sums FETCH_SIZE x 2 (the gfx950 wide-read correction, MI355X_MICROARCH.md) +
WRITE_SIZE over every adsp:: kernel of the run and divides by the number of
calls, counted as launches of the call's first kernel: k_corr_split0 (the
split form at N = 2^24) or k_absmax2 (one per call otherwise).  Also per kernel
variant (template arguments kept).  bench.py quotes the per-call figure only
for the same n."""
import csv
import json
import sys
from collections import defaultdict

root = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 23


def load(kind):
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in csv.DictReader(open(f"{root}/pmc_{kind}/corr_counter_collection.csv")):
        name = r["Kernel_Name"]
        if "adsp::" not in name:
            continue
        k = name.split("(")[0].replace("void ", "")
        tot[k] += float(r["Counter_Value"]) * 1024.0
        cnt[k] += 1
    return tot, cnt


ft, fc = load("fetch")
wt, wc = load("write")
calls = sum(v for k, v in fc.items() if "k_corr_split0" in k) or sum(v for k, v in fc.items() if "k_absmax2" in k)
out = {"per_kernel": {}}
total = 0.0
for k in ft:
    b = 2.0 * ft[k] + wt.get(k, 0.0)
    total += b
    out["per_kernel"][k] = {"hbm_bytes_per_call": round(b / calls), "launches_per_call": fc[k] / calls}
out["hbm_bytes_per_call"] = round(total / calls)
out["calls"] = calls
out["_config"] = {"workload": "corr", "n": n}
out["note"] = "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes, per CorrelateFFT call"
print(json.dumps(out, indent=1))
