#!/bin/bash
# Per-kernel averages (rocprofv3 --kernel-trace --stats) of bench.py --workload fx
# for each library build in LIBS (.so paths; "-" = in-tree), e.g. builds with
# -DAD_FX_TP_SERIAL where every stage runs alone on one stream (isolated times).
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
i=0
for v in ${LIBS:-"-"}; do
  i=$((i+1))
  if [ "$v" = "-" ]; then L=$R/algo-dsp_amd/libalgodsp_hip.so; else L=$R/$v; fi
  ALGODSP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fxiso_$i -o fx \
      -- python3 $R/bench.py --workload fx --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/fxiso_$i.json 2>/dev/null || { echo "rocprof $v failed"; exit 1; }
  python3 - "$R/gpurun_out/fxiso_$i" "$v" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + '/**/fx_kernel_stats.csv', recursive=True)[0]
d = json.loads(open(sys.argv[1] + '.json').read().strip().splitlines()[-1])
print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'])
for r in csv.DictReader(open(f)):
    if float(r['AverageNs']) > 20000:
        print(f"   {r['Name'][:58]:58s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
done
