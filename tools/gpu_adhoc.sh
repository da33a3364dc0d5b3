set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dsp_gpu.py tests/test_fxgraph.py -p no:cacheprovider > gpurun_out/t_fx.log 2>&1; rc=$?; tail -3 gpurun_out/t_fx.log; [ $rc -eq 0 ] || exit $rc
for g in "" "--graph config5" "--graph branched"; do
timeout -k 10 200 python bench.py --workload fx --steps 3 --warmup 1 --no-cpu-baseline $g > gpurun_out/bfx.log 2>&1 || { tail -5 gpurun_out/bfx.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bfx.log
done
