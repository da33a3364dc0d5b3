#!/bin/bash
# Round-4 A/B batch: spectral GPU tests, fused-vs-unfused CorrelateFFT bit
# check, CorrelateFFT A/B (unfused / default / absmax unroll-8), shard A/B
# (mix kernel with B loads ahead of A's transform vs default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_spectral_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_t_spec.log 2>&1 || { tail -30 gpurun_out/r04_t_spec.log; exit 1; }
tail -2 gpurun_out/r04_t_spec.log
timeout -k 10 300 python -u tools/corr_fused_check.py > gpurun_out/r04_corr_fused_check.txt 2>&1; cat gpurun_out/r04_corr_fused_check.txt
CORR_VARIANTS="ab/corr_unfused.so - ab/absmax_u8.so ab/fft_fwx1.so ab/corr_unfused.so - ab/absmax_u8.so ab/fft_fwx1.so" timeout -k 10 400 bash tools/corr_ab.sh > gpurun_out/r04_corr_ab.txt 2>&1; cat gpurun_out/r04_corr_ab.txt
timeout -k 10 500 bash tools/shard_ab.sh > gpurun_out/r04_shard_ab.txt 2>&1; cat gpurun_out/r04_shard_ab.txt
