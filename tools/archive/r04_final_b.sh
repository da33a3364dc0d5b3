#!/bin/bash
# Round-4 final evidence, part B: spectral parity of the final build, then
# rocprofv3 kernel trace + stats and separate FETCH_SIZE / WRITE_SIZE passes
# for the N = 1 bench workload and for CorrelateFFT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_fb_spec.log 2>&1 || { tail -40 gpurun_out/r04_fb_spec.log; exit 1; }
echo "spectral $(tail -1 gpurun_out/r04_fb_spec.log)"
SKIP_PMC=0 TAG=r04 bash tools/gpu_profile.sh || exit 1
TAG=r04 bash tools/gpu_corr_prof.sh || exit 1
cat gpurun_out/corrprof_r04/corr_pmc_traffic.json | head -c 600
