set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dsp_gpu.py -k "decode or irlib" -p no:cacheprovider > gpurun_out/t_dec.log 2>&1; rc=$?; tail -5 gpurun_out/t_dec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/rows_bench.py > gpurun_out/rows.log 2>&1; rc=$?; grep -o '"row": "[^"]*\|"value": [0-9.]*\|"frac": [0-9.]*' gpurun_out/rows.log | paste -sd' ' | sed 's/"row"/\n"row"/g'; exit $rc
