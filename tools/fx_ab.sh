#!/bin/bash
# Same-box A/B of config 5 (bench.py --workload fx) between library builds:
# FX_VARIANTS="ab/x.so - ab/x.so -" ("-" = the default); the variants' effect
# chain tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${FX_VARIANTS:-ab/fx_serial_tail.so}; do
  [ "$v" = "-" ] && continue
  ALGODSP_LIB=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_dsp_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "time_parallel or config5 or staged or engine or effect_chain" > gpurun_out/fx_ab_t.log 2>&1 || { echo "tests fail $v"; tail -20 gpurun_out/fx_ab_t.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/fx_ab_t.log)"
done
for v in ${FX_VARIANTS:-ab/fx_serial_tail.so - ab/fx_serial_tail.so -}; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  ALGODSP_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload fx --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fx_ab.json 2>/dev/null || { echo fail $v; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/fx_ab.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
