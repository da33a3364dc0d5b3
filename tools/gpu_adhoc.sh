set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dsp_gpu.py tests/test_fxgraph.py -p no:cacheprovider > gpurun_out/t_fx.log 2>&1; rc=$?; tail -3 gpurun_out/t_fx.log; [ $rc -eq 0 ] || exit $rc
for g in "" "--graph config5" "--graph branched"; do
timeout -k 10 200 python bench.py --workload fx --steps 3 --warmup 1 --no-cpu-baseline $g > gpurun_out/bfx.log 2>&1 || { tail -5 gpurun_out/bfx.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bfx.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pfx -o fx -- python3 bench.py --workload fx --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pfx.log 2>&1 || { tail -5 gpurun_out/pfx.log; exit 1; }
f=$(find gpurun_out/pfx -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
for r in csv.DictReader(open('$f')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')"
