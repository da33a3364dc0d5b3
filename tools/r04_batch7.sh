#!/bin/bash
# Round-4 batch 7: CorrelateFFT with the max-abs folded into the first pass
# (k_corr_split0 + k_fft_pass_pf PACKIN): spectral parity incl. the 2^24
# plan, the difference against the unsplit build, A/B (40 calls per run), and
# a kernel trace of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b7_spec.log 2>&1 || { tail -40 gpurun_out/r04_b7_spec.log; exit 1; }
echo "default $(tail -1 gpurun_out/r04_b7_spec.log)"
timeout -k 10 300 python -u tools/corr_fused_check.py ab/nosplit.so > gpurun_out/r04_split_check.txt 2>&1; cat gpurun_out/r04_split_check.txt
V="ab/nosplit.so - ab/split_g1024.so ab/pf0.so"
CORR_STEPS=40 CORR_VARIANTS="$V $V" timeout -k 10 600 bash tools/corr_ab.sh > gpurun_out/r04_corr_ab5.txt 2>&1 || { cat gpurun_out/r04_corr_ab5.txt; exit 1; }
cat gpurun_out/r04_corr_ab5.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/splitprof -o corr -- python3 bench.py --workload corr --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/splitprof.log 2>&1 || { tail gpurun_out/splitprof.log; exit 1; }
find gpurun_out/splitprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r04_split_kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r04_split_kernel_stats.csv')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))"
