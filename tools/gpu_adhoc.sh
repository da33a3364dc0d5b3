set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "segments" -p no:cacheprovider > gpurun_out/t3.log 2>&1; rc=$?; tail -5 gpurun_out/t3.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b3a.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --segments 4 > gpurun_out/b3b.log 2>&1 || exit $?
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --steps 5 --warmup 2 --no-cpu-baseline --mixdown on > gpurun_out/b3c.log 2>&1 || exit $?
for f in b3a b3b b3c; do grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": 5, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/$f.log; done
