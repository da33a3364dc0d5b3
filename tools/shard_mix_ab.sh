cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in "--mixdown on" "--mixdown on --pipeline off" "--mixdown off" "--mixdown on"; do
  timeout -k 10 200 python3 bench.py --workload shard --steps 20 --warmup 5 --no-cpu-baseline --clock-settle 20 $v > gpurun_out/sh.json 2>/dev/null || { echo fail "$v"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sh.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('mixdown_reduce',{}).get('conv_ms_per_step'), d.get('mixdown_reduce',{}).get('reduce_ms'))" "$v"
done
