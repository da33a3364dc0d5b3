#!/bin/bash
# Same-box sweep of the conv engine's offline schedule (ad_conv_multi_set_schedule):
# each entry of SWEEP is "serial", "pipelined:CHUNK:RUN" or "chunked:CHUNK:RUN" (0 = auto), run as a
# short bench.py each (BENCH_ARGS appended, e.g. "--workload shard"); prints
# value, ms/step, parity and the per-kernel averages.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in ${SWEEP:-"serial pipelined:0:0"}; do
  i=$((i+1))
  IFS=: read -r mode chunk run <<< "$v"
  extra="--schedule $mode"
  [ "$mode" != "serial" ] && extra="$extra --pipe-chunk ${chunk:-0} --pipe-run ${run:-0}"
  timeout -k 10 200 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --host-io off --shard-sub off \
      $extra ${BENCH_ARGS:-} > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/sweep_$i.err; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['parity']['rms'], {k:round(x['avg_us'],1) for k,x in d['kernels'].items()})" gpurun_out/sweep_$i.json "$v"
done
