#!/bin/bash
# Round-2 GPU session: parity tests, the default bench line, the config-4
# shard line and extra bench variants (BENCH_VARIANTS: ';'-separated arg sets).
# Every GPU step is bounded and the script stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  KARGS=()
  if [ -n "${PYTEST_K:-}" ]; then KARGS=(-k "$PYTEST_K"); fi
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 180 --timeout-method thread "${KARGS[@]}" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
i=0
IFS=';' read -ra VARS <<< "${BENCH_VARIANTS:-}"
for v in "${VARS[@]}"; do
  [ -z "$v" ] && continue
  i=$((i+1))
  timeout -k 10 240 python -u bench.py --no-cpu-baseline $v > gpurun_out/var_$i.json 2> gpurun_out/var_$i.err
  rc=$?; echo "variant [$v] rc=$rc"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d.get('parity',{}).get('rms'), {k:(round(x['avg_us'],1)) for k,x in d['kernels'].items()})" gpurun_out/var_$i.json 2>/dev/null || tail -3 gpurun_out/var_$i.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
