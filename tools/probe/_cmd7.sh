timeout -k 10 300 python tools/lib_ab.py 65536 tools/_build/ref_r2.so tools/_build/var_noctl.so tools/_build/var_prio1.so tools/_build/var_prio2.so > gpurun_out/ab_prio65k.txt 2>&1; echo ab65 rc=$?; cat gpurun_out/ab_prio65k.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -m gpu -x -q -s --timeout 400 --timeout-method thread -k "config3" > gpurun_out/pt_l3.log 2>&1; echo pt rc=$?; grep -E "^\[x3|passed|failed" gpurun_out/pt_l3.log
timeout -k 10 600 bash tools/x3_ab.sh old new > gpurun_out/x3_ab.txt 2>&1; echo ab rc=$?; cat gpurun_out/x3_ab.txt
