#!/bin/bash
# Config-5 A/B of library builds (LIBS: .so paths, "-" = in-tree), interleaved
# ROUNDS times: bench.py --workload fx value and ms/step per build, then a
# rocprofv3 kernel trace of the in-tree build's fx step (per-kernel averages to
# gpurun_out/fx_det_prof/).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-"-"}; do
    if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
    ALGODSP_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --workload fx --steps ${STEPS:-10} --warmup 3 \
        --no-cpu-baseline > gpurun_out/fxab.json 2> gpurun_out/fxab.err || { echo "lib $v failed"; tail -5 gpurun_out/fxab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['engine'], d['parity'] and d['parity']['rms'])" gpurun_out/fxab.json "$v"
  done
done
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fx_det_prof -o fx \
      -- python3 $GRAFT_REPO_ROOT/bench.py --workload fx --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
  python3 - <<'PY'
import csv, glob
f = glob.glob('/root/repo/gpurun_out/fx_det_prof/**/fx_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
fi
