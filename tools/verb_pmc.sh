#!/bin/bash
# SQ counters of the config-5 Freeverb kernel (one pass; isolated stages when
# $1 is a serial A/B build, e.g. ab/gser.so from tools/build_variant.sh).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/verb_pmc
mkdir -p $O
ALGODSP_LIB=$PWD/${1:-algo-dsp_amd/libalgodsp_hip.so} timeout -s KILL 120 rocprofv3 --kernel-include-regex k_fxtp_verb \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d $O -o verb --output-format csv -- python3 bench.py --workload fx --steps 1 --warmup 1 --no-cpu-baseline > $O/bench.json
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open('gpurun_out/verb_pmc/verb_counter_collection.csv')):
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(acc): print(k, acc[k] / max(1, n[k]) * 1, n[k])
PY
