timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/pt_all.log 2>&1
r=$?; echo pytest rc=$r; grep -E "seed|passed|failed|FAILED|Error" gpurun_out/pt_all.log | tail -40
if [ $r -le 1 ]; then timeout -k 10 400 python tools/probe/ab_lanes.py 1 1048576,4194304 tools/_build/var_gw6.so tools/_build/var_gw7.so tools/_build/var_gw8.so > gpurun_out/ab_gw.txt 2>&1; echo ab rc=$?; cat gpurun_out/ab_gw.txt; fi
