#!/bin/bash
# Same-box A/B of the headline bench line between trees (each a full repo copy
# with its own built library; "." is this tree): ROUNDS alternations, prints
# value and ms/step of each run.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in $(seq ${ROUNDS:-3}); do
  for t in ${TREES:-abx/r04tree .}; do
    (cd $t && timeout -k 10 200 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --host-io off --shard-sub off ${BENCH_ARGS:-}) \
      > gpurun_out/hab.json 2> gpurun_out/hab.err || { echo "fail $t"; tail -5 gpurun_out/hab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/hab.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], {k:round(x['avg_us'],1) for k,x in d.get('kernels',{}).items()})" "$t"
  done
done
