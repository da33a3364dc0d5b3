#!/bin/bash
# Round-4 batch 8: timing probes of the PACKIN second pass (tools/ builds with
# wrong results, timing only): 1 = its mirror loads made contiguous, 2 = its
# stores made contiguous; against the default and the unsplit build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="ab/nosplit.so - ab/pexp1.so ab/pexp2.so"
for v in $V $V; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 120 python bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/corr.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/corr.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done | tee gpurun_out/r04_packin_probe.txt
