# round-4 GPU call: full-batch parity diagnostics, the large-batch form sweep, the learner A/B
# (tools/_build/x3_old.so vs x3_new.so: gradient bits, alternating timing) and the learner tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4_full 300 python -u -m pytest tests/test_gpu_parity_full.py -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "step_matches or rollout_first or traj_ctbr"
step r4_x3_bits 300 python -u tools/x3_bits_ab.py tools/_build/x3_old.so tools/_build/x3_new.so
step r4_x3_time 500 bash tools/x3_ab_time.sh
step r4_learner_tests 400 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_sb3_vec_env.py tests/test_gpu_train.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider
step r4_dram_sweep 400 python -u tools/dram_sweep.py
echo "=== done"
