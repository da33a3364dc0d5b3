#!/bin/bash
# Round-6 evidence: the whole GPU suite, smoke(), the default bench line (N = 1
# with its legs), the CorrelateFFT line, then rocprofv3 kernel trace + stats and
# separate FETCH_SIZE / WRITE_SIZE passes for the headline and for CorrelateFFT.
# Every GPU step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06}
if [ "${SKIP_SUITE:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/${T}_pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
fi
t0=$(date +%s.%N)
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
echo "bench wall s: $(python3 -c "import sys; print(round(float(sys.argv[2]) - float(sys.argv[1]), 1))" $t0 $(date +%s.%N))"
tail -c 300 gpurun_out/${T}_bench.json; echo
timeout -k 10 300 python3 -u bench.py --workload corr --steps 40 --warmup 3 > gpurun_out/${T}_corr_bench.json 2> gpurun_out/${T}_corr_bench.err || { tail gpurun_out/${T}_corr_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_corr_bench.json; echo
TAG=$T bash tools/gpu_profile.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_$T > gpurun_out/prof_$T/pmc_traffic.json || exit 1
TAG=$T bash tools/gpu_corr_prof.sh || exit 1
echo final done
