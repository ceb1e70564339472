# round-4 GPU call: rollout actor-W2-in-LDS A/B + bit identity + rollout tests; DRAM A/B; parity
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 40 "gpurun_out/$name.log" | grep -v amdgpu.ids
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4_digest2 400 python -u tools/env_digest.py tools/_build/ref_prev.so uav_reinforcement_learning_control_amd/_lib/libquadenv.so
step r4_roll_ab 500 python -u tools/rollout_variants.py 65536 64
step r4_rtests 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_policy.py tests/test_gpu_parity_full.py -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider
step r4_dram_ab 700 bash tools/dram_ab.sh tools/_build/var_w6.so 4194304,8388608 1,2,0n 3
echo "=== done"
