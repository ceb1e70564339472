# A/B tool (not product): quad_ppo_grad at 524,288 rows for the in-tree-style build x3_new.so at
# several actor shares (QUADENV_X3_ACTOR_SHARE), with x3_old.so as the reference between them.
# usage: bash tools/x3_share_sweep.sh [shares...]
set -u
shares=${*:-500 520 540 560 580}
echo "== old"; QUADENV_LIB=tools/_build/x3_old.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
for sh in $shares; do
  echo "== new share $sh"; QUADENV_X3_ACTOR_SHARE=$sh QUADENV_LIB=tools/_build/x3_new.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
done
echo "== old"; QUADENV_LIB=tools/_build/x3_old.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
