# A/B tool (not product): quad_ppo_grad variants tools/_build/x3_<name>.so -- the gradient bits of
# each (tools/x3_bits_ab.py), then learner_bench at 524,288 rows, the names in turn, twice.
# Usage: x3_ab4.sh name1 name2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
libs=""; for n in "$@"; do libs="$libs tools/_build/x3_$n.so"; done
timeout -k 10 600 python -u tools/x3_bits_ab.py $libs || exit 1
for rep in 1 2; do
  for n in "$@"; do
    echo "== $n"; QUADENV_LIB=tools/_build/x3_$n.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
  done
done
