#!/bin/bash
# Same-box A/B of whole library builds: each entry of LIBS is a .so path
# ("-" = the in-tree algo-dsp_amd/libalgodsp_hip.so), run as a short bench.py
# each (BENCH_ARGS appended; default the conv headline without the extra legs),
# interleaved ROUNDS times; prints value, ms/step and the kernel averages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-"-"}; do
    if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
    ALGODSP_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline \
        --host-io off --shard-sub off --fx-leg off --stream-leg off ${BENCH_ARGS:-} > gpurun_out/libab.json 2> gpurun_out/libab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "lib $v rc=$rc"; tail -5 gpurun_out/libab.err; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], 'settled', (d.get('settled') or {}).get('median_ms_last_half'), {k:round(x['avg_us'],1) for k,x in d.get('kernels',{}).items()})" gpurun_out/libab.json "$v"
  done
done
