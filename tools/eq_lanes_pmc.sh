#!/bin/bash
# SQ counters of K_lanes (k_fx_eq_lanes) at 256 ch x 2^20, two passes, for the
# default build and (LN_PMC_VARIANT, an abx/*.so) a probe build beside it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/eq_lanes_pmc
mkdir -p $OUT
for v in - ${LN_PMC_VARIANT:-}; do
  if [ "$v" = "-" ]; then L=$PWD/algo-dsp_amd/libalgodsp_hip.so; t=def; else L=$PWD/$v; t=$(basename $v .so); fi
  ALGODSP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --output-format csv -d $OUT/${t}_p1 -o p -- python3 tools/eq_lanes_once.py > $OUT/${t}_log1 2>&1 || { tail $OUT/${t}_log1; exit 1; }
  ALGODSP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM \
    --output-format csv -d $OUT/${t}_p2 -o p -- python3 tools/eq_lanes_once.py > $OUT/${t}_log2 2>&1 || { tail $OUT/${t}_log2; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob('gpurun_out/eq_lanes_pmc/*_p*/p_counter_collection.csv')):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if 'eq_lanes' not in r['Kernel_Name']:
            continue
        acc[r['Dispatch_Id']][r['Counter_Name']].append(float(r['Counter_Value']))
    last = sorted(acc, key=int)[-1]
    print(f, 'dispatch', last)
    for c in sorted(acc[last]): print('   ', c, sum(acc[last][c]))
PY
