#!/bin/bash
# Round-4 final check of the committed build: the whole GPU suite, smoke(),
# and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_pytest_gpu_final.log 2>&1 || { tail -40 gpurun_out/r04_pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/r04_pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04_bench_final.json 2> gpurun_out/r04_bench_final.err || { tail gpurun_out/r04_bench_final.err; exit 1; }
tail -c 300 gpurun_out/r04_bench_final.json; echo
timeout -k 10 300 python3 -u bench.py --workload corr --steps 40 --warmup 3 > gpurun_out/r04_corr_bench_final.json 2>/dev/null || exit 1
tail -c 200 gpurun_out/r04_corr_bench_final.json; echo
