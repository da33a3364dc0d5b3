#!/bin/bash
# CorrelateFFT plan order A/B (AD_FFT_ENDS: the half inverse as 256.128.256
# instead of 256.256.128): spectral tests on the variant, then two interleaved
# rounds of bench.py --workload corr per build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALGODSP_LIB=$PWD/abx/ends.so timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/corr_ends_t.log 2>&1 || { tail -20 gpurun_out/corr_ends_t.log; exit 1; }
tail -1 gpurun_out/corr_ends_t.log
for r in 1 2; do
  for v in - abx/ends.so; do
    if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
    o=$(ALGODSP_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    echo "$v $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'])" "$o")"
  done
done
