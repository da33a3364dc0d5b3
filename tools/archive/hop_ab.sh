#!/bin/bash
# Same-box A/B of the headline at several hops (HOPS), ROUNDS interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for h in ${HOPS:-8192 4096}; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io off --shard-sub off \
        --fx-leg off --stream-leg off --hop $h > gpurun_out/hopab.json 2> gpurun_out/hopab.err || { echo "hop $h failed"; tail -5 gpurun_out/hopab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('hop', sys.argv[2], d['value'], d['ms_per_step'], 'settled', (d.get('settled') or {}).get('median_ms_last_half'), d['parity']['rms'], {k:round(x['avg_us'],1) for k,x in d.get('kernels',{}).items()})" gpurun_out/hopab.json "$h"
  done
done
