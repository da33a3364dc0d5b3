#!/bin/bash
# Round-4 batch 10: the split first pass with 16-B LDS staging of column pairs
# and a branch-light stage-out (default) against the previous split build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b10_spec.log 2>&1 || { tail -40 gpurun_out/r04_b10_spec.log; exit 1; }
echo "default $(tail -1 gpurun_out/r04_b10_spec.log)"
V="- ab/split.so ab/nosplit.so"
for v in $V $V; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 120 python bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/corr.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/corr.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done | tee gpurun_out/r04_split_ab2.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/splitprof2 -o corr -- python3 bench.py --workload corr --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/splitprof2.log 2>&1 || { tail gpurun_out/splitprof2.log; exit 1; }
find gpurun_out/splitprof2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r04_split_kernel_stats2.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r04_split_kernel_stats2.csv')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))"
