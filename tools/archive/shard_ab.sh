#!/bin/bash
# Same-box A/B of the shard workload (bench.py --workload shard) between
# library builds: SHARD_VARIANTS="ab/x.so - ab/x.so -" ("-" = the default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${SHARD_VARIANTS:-ab/k3mix_ab.so - ab/k3mix_v16.so ab/k3mix_v16ab.so ab/k3mix_ab.so - ab/k3mix_v16.so ab/k3mix_v16ab.so}; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload shard --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/shard_ab.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/shard_ab.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], {k: round(x['avg_us'],1) for k, x in d['kernels'].items()}, d['parity']['rms'])"
done
