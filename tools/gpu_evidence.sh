#!/bin/bash
# Refresh every committed measurement in one GPU session: parity tests, the
# headline bench line, its rocprofv3 kernel stats and PMC traffic passes,
# the per-row measurements, the config-4 shard, config-5, streaming and
# correlation bench lines.  Each step is time-limited; the script stops at
# the first failure.  Outputs: gpurun_out/ev_* (copied to profiles/ by hand).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ev_pytest.log 2>&1 || { tail -30 gpurun_out/ev_pytest.log; exit 1; }
tail -2 gpurun_out/ev_pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err || { tail gpurun_out/ev_bench.err; exit 1; }
tail -1 gpurun_out/ev_bench.json | cut -c1-300
TAG=$TAG bash tools/gpu_profile.sh > gpurun_out/ev_profile.log 2>&1 || { tail gpurun_out/ev_profile.log; exit 1; }
timeout -k 10 300 python bench.py --workload shard --steps 10 --warmup 3 --no-cpu-baseline --host-io off > gpurun_out/ev_shard.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload fx --steps 3 --warmup 1 > gpurun_out/ev_fx.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload stream --steps 3 --warmup 1 > gpurun_out/ev_stream.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload corr --steps 5 --warmup 2 > gpurun_out/ev_corr.json 2>/dev/null || exit 1
TAG=$TAG bash tools/gpu_corr_prof.sh > gpurun_out/ev_corrprof.log 2>&1 || { tail gpurun_out/ev_corrprof.log; exit 1; }
bash tools/fx_prof.sh > gpurun_out/ev_fxprof.log 2>&1 || { tail gpurun_out/ev_fxprof.log; exit 1; }
timeout -k 10 500 python -u tools/rows_bench.py --out gpurun_out/ev_rows.json > gpurun_out/ev_rows.log 2>&1 || { tail gpurun_out/ev_rows.log; exit 1; }
echo done
