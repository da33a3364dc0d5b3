#!/bin/bash
# A/B of kernel variants selected by environment: each VARIANT is
# "ENV=V[,ENV=V...]" (or "-" for the default), run as a short bench each;
# prints value, ms/step and per-kernel averages.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in ${VARIANTS:-"-"}; do
  i=$((i+1))
  envs=""
  [ "$v" != "-" ] && envs=${v//,/ }
  env $envs timeout -k 10 200 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --host-io off \
      ${BENCH_ARGS:-} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/ab_$i.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['parity']['rms'], {k:round(x['avg_us'],1) for k,x in d['kernels'].items()})" gpurun_out/ab_$i.json "$v"
done
