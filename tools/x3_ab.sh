# A/B of learner builds (tools/_build/x3_<name>.so): quad_ppo_grad at 524,288 rows, alternating
# usage: bash tools/x3_ab.sh old new   (default: old new)
set -u
a=${1:-old}; b=${2:-new}
for v in $a $b $a $b $a $b; do
  echo "== $v"; QUADENV_LIB=tools/_build/x3_$v.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
done
