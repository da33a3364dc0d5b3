"""Per-kernel HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Usage: python tools/pmc_traffic.py <prof_dir> [channels samples hop] > profiles/pmc_traffic.json

The per-GPU workload the passes ran (default: bench.py's N = 1 config, 2
channels x 2^24 samples, hop 8192) is recorded under "_config"; bench.py
quotes the traffic only for a run of that same workload.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE on gfx950 reports
half the bytes of wide (16 B/lane) coalesced streaming reads, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both counters are in
KiB.  Launches shorter than 20 % of the kernel's median duration (the
create-time IR-spectrum launch of K1) are excluded.
"""
import csv
import json
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]


def short(name):
    base = name.split("(")[0].replace("void ", "")
    base = base.split("::")[-1]
    return base.split("<")[0]


def load(kind):
    rows = defaultdict(list)
    for r in csv.DictReader(open(f"{root}/pmc_{kind}/bench_counter_collection.csv")):
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        rows[short(r["Kernel_Name"])].append((dur, float(r["Counter_Value"]) * 1024.0))
    return rows


fetch, write = load("fetch"), load("write")
out = {}
for k in fetch:
    if k.startswith("__amd"):
        continue
    med = statistics.median(d for d, _ in fetch[k])
    f = [v for d, v in fetch[k] if d >= 0.2 * med]
    med_w = statistics.median(d for d, _ in write.get(k, [(1, 0)]))
    w = [v for d, v in write.get(k, []) if d >= 0.2 * med_w]
    fb = 2.0 * sum(f) / len(f)
    wb = sum(w) / len(w) if w else 0.0
    out[k] = {
        "hbm_bytes_per_launch": round(fb + wb),
        "read_bytes_per_launch": round(fb),
        "write_bytes_per_launch": round(wb),
        "launches": len(f),
        "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes",
    }
cfg = [int(v) for v in sys.argv[2:5]] if len(sys.argv) >= 5 else [2, 1 << 24, 8192]
out["_config"] = {"channels": cfg[0], "samples": cfg[1], "hop": cfg[2]}
print(json.dumps(out, indent=1))
