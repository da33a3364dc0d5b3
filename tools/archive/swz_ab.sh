#!/bin/bash
# A/B of the linear LDS-swizzle split (fft_device.hpp lds_slot_split) against
# abx/old.so: bit-identity of the headline step's output and of CorrelateFFT,
# then interleaved bench rounds (headline and CorrelateFFT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/swz_identity.py algo-dsp_amd/libalgodsp_hip.so abx/old.so || exit 1
for r in 1 2; do
  for v in - abx/old.so; do
    if [ "$v" = "-" ]; then L=algo-dsp_amd/libalgodsp_hip.so; else L=$v; fi
    h=$(ALGODSP_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io off --shard-sub off 2>/dev/null | tail -1) || exit 1
    c=$(ALGODSP_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --workload corr --steps 40 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    echo "$v headline $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['roofline']['avg_launch_us'])" "$h") corr $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'])" "$c")"
  done
done
