# kernel trace of the C streaming harness at config 2 (per-block kernel durations and gaps)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/strace
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/strace -o st --output-format csv -- ./tools/stream_bench 16384 4096 1000 ols > gpurun_out/strace/bench.json
find gpurun_out/strace -name "*.csv" | head
