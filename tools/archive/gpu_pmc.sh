#!/bin/bash
# One rocprofv3 PMC pass per counter group over a short bench run (kernel
# trace only; never combined with sys/runtime tracing).  PMC="A B,C D" runs
# one pass per space-separated group (commas join counters in one pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
BARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --kernel-timing off}
i=0
for grp in ${PMC:-"SQ_WAIT_ANY,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_ANY"}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${grp//,/ } --output-format csv -d $OUT/p$i -o bench -- python3 bench.py $BARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT
