#!/bin/bash
# K_lanes A/B on one box: the bit-exact tests of the default build, then the
# 256 ch x 2^20 call time of each variant (LN_VARIANTS, "-" = the default;
# abx/*.so built by tools/build_variant.sh with AD_LN_EXP probe flags).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dsp_gpu.py -x -q --timeout 120 --timeout-method thread -k "eq_lanes or eq_only or staged_engine_matches_fused or noise_guard or biquad or chain" > gpurun_out/eqlanes_tests.log 2>&1
rc=$?; tail -2 gpurun_out/eqlanes_tests.log; [ $rc = 0 ] || exit $rc
for v in ${LN_VARIANTS:--}; do
  if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
  echo "$v $(ALGODSP_LIB=$PWD/$L timeout -k 10 120 python tools/eq_lanes_time.py 2>&1 | grep -v amdgpu.ids)" || exit 1
done
