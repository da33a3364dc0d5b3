# kernel statistics of the config-5 bench with the library in $1 (ALGODSP_LIB)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fxprof_$(basename $1 .so)
mkdir -p $O
ALGODSP_LIB=$PWD/$1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o fx --output-format csv -- python3 bench.py --workload fx --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json
python3 -c "
import csv,json
for r in csv.DictReader(open('$O/fx_kernel_stats.csv')): print(r['Name'][29:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
print(json.loads(open('$O/bench.json').read().strip().splitlines()[-1])['value'])
"
