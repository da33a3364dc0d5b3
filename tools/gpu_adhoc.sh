set -u
cp algo-dsp_amd/libalgodsp_hip.so /tmp/base.so
for v in base nt nt2 base nt nt2; do
  case $v in nt) cp algo-dsp_amd/libalgodsp_hip_nt.so algo-dsp_amd/libalgodsp_hip.so;; nt2) cp algo-dsp_amd/libalgodsp_hip_nt2.so algo-dsp_amd/libalgodsp_hip.so;; *) cp /tmp/base.so algo-dsp_amd/libalgodsp_hip.so;; esac
  echo "$v $(timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k:round(v["avg_us"],1) for k,v in d["kernels"].items()})')"
done
cp /tmp/base.so algo-dsp_amd/libalgodsp_hip.so
