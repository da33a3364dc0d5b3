#!/bin/bash
# Round-4 batch 12: the fused forward-last / inverse-first CorrelateFFT kernel
# at 1024 threads (8 inverse pairs, 128-B input runs, one workgroup per CU;
# all waves busy in both halves since the 4-value inverse) against 512.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALGODSP_LIB=$PWD/ab/fused1024.so timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b12_spec.log 2>&1 || { tail -40 gpurun_out/r04_b12_spec.log; exit 1; }
echo "fused1024 $(tail -1 gpurun_out/r04_b12_spec.log)"
V="- ab/fused1024.so"
for v in $V $V $V; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 120 python bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/corr.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/corr.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done | tee gpurun_out/r04_fused_nt_ab.txt
