# streaming tests (incl. the pre-enqueued chain paths), then C-harness block latencies
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "stream or config2" > gpurun_out/r03_gate_tests.log 2>&1 || { tail -30 gpurun_out/r03_gate_tests.log; exit 1; }
tail -3 gpurun_out/r03_gate_tests.log
for cfg in "16384 4096 4096" "16384 2048 4096" "131072 4096 2048" "131072 8192 2048"; do
  timeout -k 10 60 ./tools/stream_bench $cfg ols
done | tee gpurun_out/r03_stream_c2.jsonl
