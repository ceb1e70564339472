# round-4 GPU call: k_rollout built with the backend's max-ilp / max-memory-clause scheduling -- bits
# (every step form and the rollout) vs the in-tree build, then the per-step time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=uav_reinforcement_learning_control_amd/_lib/libquadenv.so
timeout -k 10 400 python -u tools/env_digest.py $L tools/_build/roll_ilp.so > gpurun_out/r4_roll_sched_bits.txt 2>&1 || { tail -5 gpurun_out/r4_roll_sched_bits.txt; exit 1; }
tail -3 gpurun_out/r4_roll_sched_bits.txt
timeout -k 10 400 python -u tools/env_digest.py $L tools/_build/roll_mem.so > gpurun_out/r4_roll_sched_bits2.txt 2>&1 || { tail -5 gpurun_out/r4_roll_sched_bits2.txt; exit 1; }
tail -3 gpurun_out/r4_roll_sched_bits2.txt
ROLL_VARIANTS=base,ilp,mem,ilp,base,mem,mem,base,ilp timeout -k 10 600 python -u tools/rollout_variants.py 65536 128 > gpurun_out/r4_roll_sched.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_roll_sched.txt
