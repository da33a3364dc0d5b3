#!/bin/bash
# CorrelateFFT evidence: kernel trace + stats and separate FETCH_SIZE /
# WRITE_SIZE passes over bench.py --workload corr (one pass per counter group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/corrprof_$TAG
mkdir -p $OUT
BARGS="--workload corr --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o corr -- python3 bench.py $BARGS > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o corr -- python3 bench.py $BARGS > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o corr -- python3 bench.py $BARGS > $OUT/write.log 2>&1 || { tail $OUT/write.log; exit 1; }
python3 tools/pmc_call_traffic.py $OUT > $OUT/corr_pmc_traffic.json || exit 1
echo corrprof done
