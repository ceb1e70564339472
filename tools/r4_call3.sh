# round-4 GPU call: parity (Euler bar), bit identity of the refactored / overlapped kernels, rollout
# A/B and ablations, waves-per-EU A/B at DRAM sizes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4_digest 400 python -u tools/env_digest.py tools/_build/ref_prev.so uav_reinforcement_learning_control_amd/_lib/libquadenv.so tools/_build/roll_OVL0.so
step r4_full2 400 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_rollout.py "tests/test_gpu_parity.py::test_kernel_form_selection" "tests/test_gpu_parity.py::test_step_matches_oracle_random_states" -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider
step r4_roll_abl 400 python -u tools/rollout_variants.py 65536 64
step r4_x3pk_bits 300 python -u tools/x3_bits_ab.py tools/_build/x3_old.so tools/_build/x3_new.so
step r4_x3pk_time 400 bash tools/x3_ab_time.sh
step r4_w6_a 300 python -u tools/dram_sweep.py 2097152,4194304 1,2
step r4_w6_b 300 env QUADENV_LIB=tools/_build/var_w6.so python -u tools/dram_sweep.py 2097152,4194304,8388608 1,2
step r4_w6_c 300 python -u tools/dram_sweep.py 4194304,8388608 2,0,0n
echo "=== done"
