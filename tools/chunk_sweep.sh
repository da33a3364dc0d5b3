#!/bin/bash
# Chunk-size sweep of the headline bench (blocks per channel per engine chunk;
# 0 = one chunk): each entry "CHUNK[:ENV=V,...]" runs a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in ${SWEEP:-"0 256 512"}; do
  i=$((i+1))
  ch=${v%%:*}; envs=""
  [ "$ch" != "$v" ] && envs=${v#*:} && envs=${envs//,/ }
  env $envs timeout -k 10 200 python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --host-io off --chunk $ch > gpurun_out/cs_$i.json 2> gpurun_out/cs_$i.err || { echo "$v failed"; tail -5 gpurun_out/cs_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['parity']['rms'], {k:(round(x['avg_us'],1), x['launches']) for k,x in d['kernels'].items()})" gpurun_out/cs_$i.json "$v"
done
