set -u
timeout -k 10 60 ./tools/stream_bench 16384 4096 2048 ols | tail -1
AD_STREAM_GRAPH=0 timeout -k 10 60 ./tools/stream_bench 16384 4096 2048 ols | tail -1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -p no:cacheprovider 2>&1 | tail -3
