#!/bin/bash
# Parity (FFT/conv/spectral GPU tests) and same-box timing of variant libraries against the default:
#   VARIANTS="abx/A.so abx/B.so" tools/variant_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  ALGODSP_LIB=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_spectral_gpu.py tests/test_conv_gpu.py tests/test_schedule_gpu.py \
      -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vc_t.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/vc_t.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/vc_t.log; exit $rc; }
done
CORR_VARIANTS="- $VARIANTS - $VARIANTS" bash tools/corr_ab.sh || exit 1
LIBS="- $VARIANTS" ROUNDS=${ROUNDS:-2} bash tools/lib_ab.sh
