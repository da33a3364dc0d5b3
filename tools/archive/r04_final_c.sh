#!/bin/bash
# Round-4 final evidence, part C (after the fused pass's workgroup change):
# the whole GPU suite, smoke(), the CorrelateFFT bench line, and its kernel
# trace + PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_pytest_gpu_final.log 2>&1 || { tail -40 gpurun_out/r04_pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/r04_pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python3 -u bench.py --workload corr --steps 40 --warmup 3 > gpurun_out/r04_corr_bench.json 2> gpurun_out/r04_corr_bench.err || { tail gpurun_out/r04_corr_bench.err; exit 1; }
tail -c 300 gpurun_out/r04_corr_bench.json; echo
TAG=r04 bash tools/gpu_corr_prof.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/corrprof_r04/corr_pmc_traffic.json')); print(d['hbm_bytes_per_call'])"
