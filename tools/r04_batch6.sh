#!/bin/bash
# Round-4 batch 6: CorrelateFFT A/B of k_fft_pass_pf's grid size and values
# per thread (8: 512-thread workgroups, 2 per CU; 4: 1024 threads, 1 per CU),
# of the max-abs grid (workgroups per signal, 4 or 8 loads in flight) and of
# the 16-B real-pair stores of the last inverse pass (rovec0: without).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b6_spec.log 2>&1 || { tail -30 gpurun_out/r04_b6_spec.log; exit 1; }
echo "default $(tail -1 gpurun_out/r04_b6_spec.log)"
timeout -k 10 300 python -u tools/corr_fused_check.py ab/rovec0.so > gpurun_out/r04_rovec_check.txt 2>&1; cat gpurun_out/r04_rovec_check.txt
V="ab/pf0.so ab/rovec0.so - ab/pf_g1024.so ab/pf_g2048.so ab/pf_v4_g256.so ab/pf_v4_g512.so ab/pf_v4_g1024.so ab/am_g512.so ab/am_g1024.so ab/am_g512u8.so ab/am_g1024u8.so"
CORR_VARIANTS="$V $V" timeout -k 10 800 bash tools/corr_ab.sh > gpurun_out/r04_corr_ab4.txt 2>&1 || { cat gpurun_out/r04_corr_ab4.txt; exit 1; }
cat gpurun_out/r04_corr_ab4.txt
for L in ab/pf_v4_g512.so ab/pf_v4_g1024.so; do
  ALGODSP_LIB=$PWD/$L timeout -k 10 200 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b6_spec.log 2>&1 || { tail -30 gpurun_out/r04_b6_spec.log; exit 1; }
  echo "$L $(tail -1 gpurun_out/r04_b6_spec.log)"
done
