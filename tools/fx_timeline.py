"""Config-5 pipeline timeline from a rocprofv3 kernel trace: per chunk, each
stage's start/end (us, relative to a detector launch in the middle of the run)
and its queue, plus per-kernel medians.

  python3 tools/fx_timeline.py <kernel_trace.csv>
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def name(r):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:30]


rows = [r for r in csv.DictReader(open(sys.argv[1])) if name(r).startswith(("k_fx", "k_vbuf"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
for r in rows:
    dur[name(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(dur.items()):
    print(f"{k:24s} n={len(v):4d} median {statistics.median(v):8.1f} us")
dets = [i for i, r in enumerate(rows) if name(r) == "k_fxtp_det"]
i0 = dets[len(dets) // 2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[max(0, i0 - 10):i0 + 30]:
    s = (int(r["Start_Timestamp"]) - t0) / 1000
    e = (int(r["End_Timestamp"]) - t0) / 1000
    print(f"{name(r)[:24]:24s} q{r['Queue_Id']:>3} {s:9.1f} {e:9.1f} {e - s:8.1f}")
