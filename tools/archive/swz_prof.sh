#!/bin/bash
# Kernel stats of the CorrelateFFT call and the headline step, default build and abx/old.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/swz
for v in - abx/old.so; do
  if [ "$v" = "-" ]; then L=$PWD/algo-dsp_amd/libalgodsp_hip.so; t=new; else L=$PWD/$v; t=old; fi
  ALGODSP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/swz/$t -o c --output-format csv -- python3 bench.py --workload corr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/swz/$t.log 2>&1 || exit 1
  ALGODSP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/swz/${t}h -o h --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-io off --shard-sub off > gpurun_out/swz/${t}h.log 2>&1 || exit 1
done
for f in gpurun_out/swz/*/*kernel_stats.csv; do echo $f; cut -d, -f1-4 $f | grep -E 'corr|fft_pass|irfft|window_rfft|fdl_mac' | head -8; done
