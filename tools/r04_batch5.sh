#!/bin/bash
# Round-4 batch 5: the persistent prefetching radix-256 pass (k_fft_pass_pf):
# spectral parity, bit-identity against a build without it, CorrelateFFT A/B
# of its grid size, and a kernel trace of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b5_spec.log 2>&1 || { tail -30 gpurun_out/r04_b5_spec.log; exit 1; }
tail -1 gpurun_out/r04_b5_spec.log
timeout -k 10 300 python -u tools/corr_fused_check.py ab/pf0.so > gpurun_out/r04_pf_check.txt 2>&1; cat gpurun_out/r04_pf_check.txt
CORR_VARIANTS="ab/pf0.so - ab/pf_g256.so ab/pf_g1024.so ab/pf0.so - ab/pf_g256.so ab/pf_g1024.so" timeout -k 10 400 bash tools/corr_ab.sh > gpurun_out/r04_corr_ab3.txt 2>&1 || { cat gpurun_out/r04_corr_ab3.txt; exit 1; }
cat gpurun_out/r04_corr_ab3.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pfprof -o corr -- python3 bench.py --workload corr --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pfprof.log 2>&1 || { tail gpurun_out/pfprof.log; exit 1; }
find gpurun_out/pfprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r04_pf_kernel_stats.csv
cut -d, -f1-4 gpurun_out/r04_pf_kernel_stats.csv | head -12
