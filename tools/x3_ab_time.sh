# A/B tool (not product): quad_ppo_grad at 524,288 rows under several library builds, alternating
# (A, B, ..., A, B, ...) so box drift shows; the learner_bench line of each run.
# Usage: x3_ab_time.sh [lib.so ...]   (default: tools/_build/x3_old.so tools/_build/x3_new.so)
set -u
[ $# -eq 0 ] && set -- tools/_build/x3_old.so tools/_build/x3_new.so
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib"; QUADENV_LIB=$lib timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
  done
done
