set -u
AD_K3_PERSIST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -p no:cacheprovider 2>&1 | tail -2
for v in 0 1 0 1; do
  echo "persist=$v $(AD_K3_PERSIST=$v timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k:round(v["avg_us"],1) for k,v in d["kernels"].items()})')"
done
