#!/bin/bash
# One GPU-box session: parity tests, then (if no fault) a short bench.
# Exit codes 0/1 from pytest are test outcomes; anything else (fault, abort,
# timeout) ends the script before another GPU step starts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -60 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-sample 4194304} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -20 gpurun_out/bench.log
exit $brc
