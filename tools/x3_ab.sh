set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread -k x3 2>&1 | tail -1
for v in old db2ones old db2ones; do
  echo "== $v"; QUADENV_LIB=tools/_build/x3_$v.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
done
