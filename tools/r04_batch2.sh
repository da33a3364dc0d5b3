#!/bin/bash
# Round-4 batch 2: partitioned / streaming GPU tests (the pre-enqueued emit),
# the low-latency and streaming rows from C, then r04_ab1.sh's A/B set.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_fxgraph.py -x -q --timeout 200 --timeout-method thread -k "partition or reverb or stream" > gpurun_out/r04_t_pc.log 2>&1 || { tail -40 gpurun_out/r04_t_pc.log; exit 1; }
tail -2 gpurun_out/r04_t_pc.log
: > gpurun_out/r04_stream_c.jsonl
for cfg in "95432 128 4096 pc 7 0" "95432 128 200 pc 7 2667" "95432 256 4096 pc 7 0" "95432 4096 1024 pc 7 0" \
           "16384 4096 4096 ols 7 0" "16384 2048 4096 ols 7 0" "16384 2048 100 ols 7 42667" "16384 480 4096 ols 7 0"; do
  timeout -k 10 60 ./tools/stream_bench $cfg >> gpurun_out/r04_stream_c.jsonl || { echo "stream_bench $cfg failed"; exit 1; }
done
cat gpurun_out/r04_stream_c.jsonl
bash tools/r04_ab1.sh
