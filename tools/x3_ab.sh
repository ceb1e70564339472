set -u
for v in old new old new old new; do
  echo "== $v"; QUADENV_LIB=tools/_build/x3_$v.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
done
