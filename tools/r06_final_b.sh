#!/bin/bash
# Round-6 evidence after K_lanes: the whole GPU suite, smoke(), the per-row
# table (profiles/r06_rows.json) and the default bench line, each step with its
# own limit, stopping at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 600 python3 -u tools/rows_bench.py --out gpurun_out/${T}_rows.json > gpurun_out/${T}_rows.log 2>&1 || { tail -20 gpurun_out/${T}_rows.log; exit 1; }
tail -3 gpurun_out/${T}_rows.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
tail -c 400 gpurun_out/${T}_bench.json; echo
echo final-b done
