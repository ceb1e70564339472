# round-4 GPU call: k_step_h with the helper storing the resetting envs (QD_H_RSTORE) -- bits vs the
# previous build (every step form and the rollout), then the A/B timing against the RSTORE=0 build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/env_digest.py tools/_build/ref_head.so uav_reinforcement_learning_control_amd/_lib/libquadenv.so > gpurun_out/r4rs_digest.txt 2>&1
echo "digest rc=$?"; tail -3 gpurun_out/r4rs_digest.txt
timeout -k 10 600 python -u tools/step_env_ab.py 65536,4096 3 rs0=tools/_build/var_rs0.so rs1=in-tree > gpurun_out/r4rs_ab.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/r4rs_ab.txt
