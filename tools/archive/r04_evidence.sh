#!/bin/bash
# Round-4 evidence on one box: the default bench line (N = 1, with host_io,
# shard_per_gpu and cpu_baseline), the config-2 streaming latency from C
# (back to back and paced like a real-time caller), and the rocprofv3 kernel
# trace + stats of the N = 1 workload.  Every GPU step has its own time limit
# and the steps are chained: the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit $?
tail -c 600 $OUT/${TAG}_bench.json
: > $OUT/${TAG}_stream_c.jsonl
for cfg in "16384 4096 4096 ols 7 0" "16384 2048 4096 ols 7 0" "16384 2048 100 ols 7 42667" "16384 4096 60 ols 7 85333" \
           "16384 480 4096 ols 7 0" "131072 4800 2048 ols 7 0" "95432 128 4096 pc 7 0" "95432 128 200 pc 7 2667"; do
  timeout -k 10 60 ./tools/stream_bench $cfg >> $OUT/${TAG}_stream_c.jsonl || exit $?
done
cat $OUT/${TAG}_stream_c.jsonl
if [ "${SKIP_TRACE:-0}" = "1" ]; then exit 0; fi
SKIP_PMC=${SKIP_PMC:-1} TAG=$TAG bash tools/gpu_profile.sh
