#!/bin/bash
# Round-4 batch 11: the split first pass's 16-B input loads (default) against
# two 8-B loads per pair (nofast) and the unsplit build; spectral parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b11_spec.log 2>&1 || { tail -40 gpurun_out/r04_b11_spec.log; exit 1; }
echo "default $(tail -1 gpurun_out/r04_b11_spec.log)"
V="- ab/nofast.so ab/nosplit.so"
for v in $V $V $V; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 120 python bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/corr.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/corr.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done | tee gpurun_out/r04_split_ab3.txt
