# kernel statistics of the config-5 bench (staged engine)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fxprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fxprof -o fx --output-format csv -- python3 bench.py --workload fx --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fxprof/bench.json
cut -d, -f1-6 gpurun_out/fxprof/fx_kernel_stats.csv
