set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dsp_gpu.py -x -q --timeout 120 --timeout-method thread -k "eq_lanes or eq_only or staged_engine_matches_fused or noise_guard or biquad or chain" > gpurun_out/eqlanes_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/eq_lanes_bench.py > gpurun_out/eqlanes_bench.log 2>&1
rc=$?
tail -5 gpurun_out/eqlanes_tests.log; cat gpurun_out/eqlanes_bench.log
exit $rc
