# same-box comparison of engine chunk sizes at the bench config (config 3)
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for ch in 0 1032 688; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --chunk $ch --no-cpu-baseline --host-io off --kernel-timing off > gpurun_out/c$ch.json
  python -c "import json,sys; d=json.load(open('gpurun_out/c$ch.json')); print('chunk $ch', d['ms_per_step'], d['value'])"
done
done
