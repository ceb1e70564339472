# A/B tool (not product): quad_ppo_grad at 524,288 rows, tools/_build/x3_old.so vs x3_new.so,
# alternating (old, new, old, new) so box drift shows; the learner_bench line of each run.
set -u
for lib in old new old new; do
  echo "== $lib"; QUADENV_LIB=tools/_build/x3_$lib.so timeout -k 10 120 python tools/learner_bench.py 524288 8388608 30 2>&1 | grep quad_ppo_grad || exit 1
done
