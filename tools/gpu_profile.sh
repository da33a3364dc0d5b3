#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats, then separate PMC
# passes for FETCH_SIZE and WRITE_SIZE (never combined with sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# the N = 1 workload alone (no shard_per_gpu / host_io sub-measurements in the
# kernel statistics or the PMC averages)
BARGS=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --host-io off --shard-sub off --fx-leg off --stream-leg off --corr-leg off}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py $BARGS > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 $OUT/bench_trace.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SKIP_PMC:-0}" = "1" ]; then exit 0; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o bench -- python3 bench.py $BARGS > $OUT/bench_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -3 $OUT/bench_fetch.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o bench -- python3 bench.py $BARGS > $OUT/bench_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; tail -3 $OUT/bench_write.log
find $OUT -name "*.csv" | head -20
exit $rc
