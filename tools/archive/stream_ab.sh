#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
i=0
for v in ${VARIANTS:-"-"}; do
  i=$((i+1))
  envs=""
  [ "$v" != "-" ] && envs=${v//,/ }
  env $envs timeout -k 10 120 python3 bench.py --workload stream --steps 3 --warmup 1 > gpurun_out/sab_$i.json 2> gpurun_out/sab_$i.err || { echo "variant $v failed"; tail -5 gpurun_out/sab_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], {k:d[k] for k in d if k in ('parity','config')})" gpurun_out/sab_$i.json "$v"
done
