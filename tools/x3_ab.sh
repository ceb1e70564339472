set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
for v in base nosb nol2 nodw2 nodh1; do
  echo "== $v"; QUADENV_LIB=tools/_build/x3_$v.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 20 2>&1 | grep quad_ppo_grad || exit 1
done
echo "== f32"; QUADENV_LEARNER=f32 timeout -k 10 120 python tools/learner_bench.py 524288 8388608 20 2>&1 | grep quad_ppo_grad || exit 1
tools/pmc/learner_pmc.sh
