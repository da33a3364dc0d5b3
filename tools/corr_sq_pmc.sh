#!/bin/bash
# SQ counters (LDS, VALU, waits) of the CorrelateFFT passes: one pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/corr_sq
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  --output-format csv -d $OUT -o corr -- python3 bench.py --workload corr --steps 2 --warmup 1 --no-cpu-baseline > $OUT/log 2>&1 || { tail $OUT/log; exit 1; }
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open('gpurun_out/corr_sq/corr_counter_collection.csv')):
    k = r['Kernel_Name'][:60]
    acc[k][r['Counter_Name']] += float(r['Counter_Value']); cnt[k][r['Counter_Name']] += 1
for k in acc:
    print(k)
    for c in sorted(acc[k]): print('   ', c, round(acc[k][c] / cnt[k][c]))
PY
