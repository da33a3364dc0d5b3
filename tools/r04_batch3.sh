#!/bin/bash
# Round-4 batch 3: CorrelateFFT profile (trace + PMC), then the evidence run
# (default bench line, streaming rows from C, rocprof trace of the N = 1 bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r04 bash tools/gpu_corr_prof.sh > gpurun_out/r04_corrprof.log 2>&1 || { tail -20 gpurun_out/r04_corrprof.log; exit 1; }
tail -2 gpurun_out/r04_corrprof.log
find gpurun_out/corrprof_r04/trace -name "*kernel_stats.csv" -exec cat {} \; | head -20
TAG=r04 bash tools/r04_evidence.sh > gpurun_out/r04_evidence.log 2>&1 || { tail -20 gpurun_out/r04_evidence.log; exit 1; }
tail -c 1500 gpurun_out/r04_bench.json
