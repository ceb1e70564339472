timeout -k 10 60 tools/_build/mfma_rounding > gpurun_out/mfma_rounding.txt 2>&1; echo diag rc=$?; cat gpurun_out/mfma_rounding.txt
timeout -k 10 300 python tools/lib_ab.py 65536 tools/_build/ref_r2.so tools/_build/var_noctl.so > gpurun_out/ab_ctl65k.txt 2>&1; echo ab65 rc=$?; cat gpurun_out/ab_ctl65k.txt
QUADENV_HELPER=0 timeout -k 10 300 python tools/lib_ab.py 65536 tools/_build/ref_r2.so > gpurun_out/ab_k_step65k.txt 2>&1; echo abk rc=$?; cat gpurun_out/ab_k_step65k.txt
