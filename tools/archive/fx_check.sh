# per-sample processor tests, then the config-5 bench line (staged engine) and its kernel stats
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dsp_gpu.py tests/test_fxgraph.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_fx_tests.log 2>&1 || { tail -30 gpurun_out/r03_fx_tests.log; exit 1; }
tail -2 gpurun_out/r03_fx_tests.log
timeout -k 10 200 python bench.py --workload fx --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03_fx_bench.json
python -c "import json; d=json.load(open('gpurun_out/r03_fx_bench.json')); print(d['value'], d['ms_per_step'], d.get('roofline'))"
