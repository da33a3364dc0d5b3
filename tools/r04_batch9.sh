#!/bin/bash
# Round-4 batch 9: the split CorrelateFFT with the PACKIN pass's stores through
# the L2 (split) or non-temporal (split_nt), against the unsplit default and
# the contiguous-store timing probe (pexp2, wrong results); parity of split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALGODSP_LIB=$PWD/ab/split.so timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b9_spec.log 2>&1 || { tail -40 gpurun_out/r04_b9_spec.log; exit 1; }
echo "split $(tail -1 gpurun_out/r04_b9_spec.log)"
V="- ab/split.so ab/split_nt.so ab/pexp2.so"
for v in $V $V; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 120 python bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/corr.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/corr.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done | tee gpurun_out/r04_split_ab.txt
