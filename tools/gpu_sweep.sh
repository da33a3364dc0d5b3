#!/bin/bash
# Parameter sweep of bench.py (hop, chunk, MAC run length R).  Each run is
# bounded; the sweep stops at the first run that does not exit cleanly.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_${TAG:-r01}.jsonl
: > $OUT
for cfg in ${SWEEP:-"4096:0:128 8192:0:128 8192:0:64 8192:0:256 8192:256:64 8192:512:64 4096:512:64"}; do
  IFS=: read hop chunk R <<< "$cfg"
  line=$(AD_MAC_R=$R timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --hop $hop --chunk $chunk 2> gpurun_out/sweep_err.log)
  rc=$?
  if [ $rc -ne 0 ]; then echo "cfg $cfg rc=$rc"; tail -5 gpurun_out/sweep_err.log; exit $rc; fi
  echo "{\"hop\":$hop,\"chunk\":$chunk,\"R\":$R,\"bench\":$line}" >> $OUT
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['ms_per_step'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" "$line" "$cfg"
done
