timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/pt_all.log 2>&1
r=$?; echo pytest rc=$r; grep -E "passed|failed|FAILED" gpurun_out/pt_all.log | tail -20; grep -E "^\[x3 seed" gpurun_out/pt_all.log
if [ $r -le 1 ]; then
  timeout -k 10 300 python tools/lib_ab.py 65536 tools/_build/ref_r2.so > gpurun_out/ab_ctl65k.txt 2>&1; echo ab65 rc=$?; cat gpurun_out/ab_ctl65k.txt
  timeout -k 10 300 python tools/lib_ab.py 4096 tools/_build/ref_r2.so > gpurun_out/ab_ctl4k.txt 2>&1; echo ab4k rc=$?; cat gpurun_out/ab_ctl4k.txt
  timeout -k 10 600 bash tools/x3_ab.sh old new > gpurun_out/x3_ab.txt 2>&1; echo ab rc=$?; cat gpurun_out/x3_ab.txt
fi
