#!/bin/bash
# Parameter sweep of bench.py.  Each config is hop:chunk:R[:ENV=V,ENV=V...]
# (R = MAC run length; extra env vars select kernel variants).  Each run is
# bounded; the sweep stops at the first run that does not exit cleanly.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_${TAG:-r02}.jsonl
: > $OUT
CFGS=${SWEEP:-"4096:0:128 8192:0:64"}
for cfg in $CFGS; do
  IFS=: read hop chunk R envs <<< "$cfg"
  envs=${envs:-}
  line=$(env AD_MAC_R=$R ${envs//,/ } timeout -k 10 200 python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline \
         --kernel-timing off --hop $hop --chunk $chunk 2> gpurun_out/sweep_err.log)
  rc=$?
  if [ $rc -ne 0 ]; then echo "cfg $cfg rc=$rc"; tail -5 gpurun_out/sweep_err.log; exit $rc; fi
  echo "{\"cfg\":\"$cfg\",\"bench\":$line}" >> $OUT
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['ms_per_step'], {k:(round(v['avg_us'],1), v['launches']) for k,v in d['kernels'].items()})" "$line" "$cfg"
done
