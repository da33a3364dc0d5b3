#!/bin/bash
# Round-4 final evidence, part A: the whole GPU suite, then the bench lines
# (default N = 1 with host_io / shard_per_gpu / cpu_baseline; CorrelateFFT;
# config 5) and the config-2 streaming latency from C.  Every GPU step has its
# own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04_pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { tail gpurun_out/r04_bench.err; exit 1; }
tail -c 400 gpurun_out/r04_bench.json; echo
timeout -k 10 300 python3 -u bench.py --workload corr --steps 40 --warmup 3 > gpurun_out/r04_corr_bench.json 2> gpurun_out/r04_corr_bench.err || { tail gpurun_out/r04_corr_bench.err; exit 1; }
tail -c 300 gpurun_out/r04_corr_bench.json; echo
timeout -k 10 300 python3 -u bench.py --workload fx --steps 5 --warmup 2 > gpurun_out/r04_fx_bench.json 2> gpurun_out/r04_fx_bench.err || { tail gpurun_out/r04_fx_bench.err; exit 1; }
tail -c 300 gpurun_out/r04_fx_bench.json; echo
: > gpurun_out/r04_stream_c_final.jsonl
for cfg in "16384 4096 4096 ols 7 0" "16384 2048 4096 ols 7 0" "16384 2048 100 ols 7 42667" "16384 4096 60 ols 7 85333" \
           "16384 480 4096 ols 7 0" "131072 4800 2048 ols 7 0" "95432 128 4096 pc 7 0" "95432 128 200 pc 7 2667"; do
  timeout -k 10 60 ./tools/stream_bench $cfg >> gpurun_out/r04_stream_c_final.jsonl || exit 1
done
echo streams done
