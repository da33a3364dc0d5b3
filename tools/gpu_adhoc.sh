set -u
B="--steps 8 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py $B --channels 8 --samples 4194304 --mixdown on > gpurun_out/b3.log 2>&1 || { tail gpurun_out/b3.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/b3.log | tr '\n' ' '; echo
timeout -k 10 300 python bench.py $B --channels 8 --samples 4194304 > gpurun_out/b2.log 2>&1 || { tail gpurun_out/b2.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/b2.log | tr '\n' ' '; echo
