#!/bin/bash
# Round-4 batch 14: four workgroups per CU for the split first pass (split8:
# 8 columns, 256 threads, 8192 max-abs partials) and for the persistent
# radix-256 passes (pf8: 8-butterfly tiles, 1024 workgroups), and 16-butterfly
# tiles for the last inverse pass (fwx1), against the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in ab/split8.so ab/pf8s8.so; do
  ALGODSP_LIB=$PWD/$L timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b14_spec.log 2>&1 || { tail -40 gpurun_out/r04_b14_spec.log; exit 1; }
  echo "$L $(tail -1 gpurun_out/r04_b14_spec.log)"
done
V="- ab/split8.so ab/pf8.so ab/pf8s8.so ab/fwx1.so"
for v in $V $V $V; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 120 python bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/corr.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/corr.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done | tee gpurun_out/r04_split8_ab.txt
