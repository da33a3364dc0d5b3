#!/bin/bash
# Round-4 batch 4: the whole GPU suite, then CorrelateFFT A/B of the fused
# kernel's workgroup size (512: 4 inverse pairs, 64-B input runs; 1024: 8 pairs,
# 128-B runs, one workgroup per CU) against the unfused passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04_pytest_gpu.log
CORR_VARIANTS="ab/corr_unfused.so - ab/corr_nt1024.so ab/corr_v4.so ab/corr_unfused.so - ab/corr_nt1024.so ab/corr_v4.so" timeout -k 10 400 bash tools/corr_ab.sh > gpurun_out/r04_corr_ab2.txt 2>&1; cat gpurun_out/r04_corr_ab2.txt
ALGODSP_LIB=$PWD/ab/corr_v4.so timeout -k 10 300 python -u -m pytest tests/test_spectral_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_t_spec_v4.log 2>&1; tail -2 gpurun_out/r04_t_spec_v4.log
FX_VARIANTS="ab/fx_serial_tail.so - ab/fx_serial_tail.so -" timeout -k 10 600 bash tools/fx_ab.sh > gpurun_out/r04_fx_ab.txt 2>&1; cat gpurun_out/r04_fx_ab.txt
