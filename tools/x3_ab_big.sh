# A/B tool (not product): quad_ppo_grad variants tools/_build/x3_<name>.so -- gradient bits, then
# learner_bench at config 3's 524,288-row minibatches drawn from a 67M-row buffer, names in turn, twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
libs=""; for n in "$@"; do libs="$libs tools/_build/x3_$n.so"; done
timeout -k 10 600 python -u tools/x3_bits_ab.py $libs || exit 1
for rep in 1 2; do
  for n in "$@"; do
    echo "== $n"; QUADENV_LIB=tools/_build/x3_$n.so timeout -k 10 200 python tools/learner_bench.py 524288 67108864 30 2>&1 | grep quad_ppo_grad || exit 1
  done
done
