#!/bin/bash
# Same-box A/B of bench.py argument sets (FLAGSETS, ';'-separated), ROUNDS interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${FLAGSETS:-}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for f in "${SETS[@]}"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io off --shard-sub off \
        --fx-leg off --stream-leg off $f > gpurun_out/flagab.json 2> gpurun_out/flagab.err || { echo "failed: $f"; tail -5 gpurun_out/flagab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(repr(sys.argv[2]), d['value'], d['ms_per_step'], (d.get('settled') or {}).get('median_ms_last_half'))" gpurun_out/flagab.json "$f"
  done
done
