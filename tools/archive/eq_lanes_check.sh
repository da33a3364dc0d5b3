cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_dsp_gpu.py tests/test_fxgraph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dsp_tests.log 2>&1; rc=$?; tail -2 gpurun_out/dsp_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/eq_lanes_bench.py 2>&1 | grep -v amdgpu
