# round-4 GPU call: k_step_h's per-step outputs (obs rows, reward, flags) written nt (A/B build) --
# the step kernel at 65,536 envs, then the bench with its two-launch rollout (the policy kernel
# reads the obs rows right after the step) under both libraries
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_env_ab.py 65536,4096 3 base=in-tree ntout=tools/_build/var_ntout.so > gpurun_out/r4_ntout_ab.txt 2>&1 || exit 1
cat gpurun_out/r4_ntout_ab.txt
for lib in in-tree ntout in-tree ntout; do
  if [ $lib = in-tree ]; then unset QUADENV_LIB; else export QUADENV_LIB=tools/_build/var_ntout.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --e2e-iters 0 > gpurun_out/r4_ntout_bench_$lib.txt 2>&1 || exit 1
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/r4_ntout_bench_$lib.txt') if x.startswith('{')][-1]); r=d['rollout_phase']
print('$lib', 'value %.4g kernel %.3f us | rollout one-launch %.4g two-launch(mfma) %.4g policy kernel %.2f us' % (d['value'], d['roofline']['kernel_us'], r['one_launch']['env_steps_per_s'], r['mfma']['env_steps_per_s'], r['policy_kernel']['kernel_us']))" | tee -a gpurun_out/r4_ntout_ab.txt
done
unset QUADENV_LIB
