set -e
mkdir -p gpurun_out
for cfg in "16384 4096 4096" "16384 480 8192" "16384 960 8192" "16384 1000 8192" "16384 4800 4096" "131072 4096 2048" "131072 480 4096" "131072 4800 2048"; do
  timeout -k 10 60 ./tools/stream_bench $cfg ols
done > gpurun_out/r03_stream_c.jsonl
cat gpurun_out/r03_stream_c.jsonl
