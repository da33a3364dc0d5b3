#!/bin/bash
# Same-box A/B of the bit-exact EQ-only chain (256 ch x 2^20, staged engine,
# per-section pipeline): EQ_VARIANTS="- abx/x.so - abx/x.so" ("-" = default);
# each variant's bit-exactness tests first, then tools/eq_waves.py per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${EQ_VARIANTS}; do
  [ "$v" = "-" ] && continue
  ALGODSP_LIB=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_dsp_gpu.py -x -q --timeout 200 --timeout-method thread -k "eq_only or staged or biquad or chain" > gpurun_out/eq_ab_t.log 2>&1 || { echo "tests fail $v"; tail -20 gpurun_out/eq_ab_t.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/eq_ab_t.log)"
done
for v in ${EQ_VARIANTS}; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  echo "$v $(ALGODSP_LIB=$PWD/$L timeout -k 10 120 python tools/eq_waves.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" || exit 1
done
