# round-4 GPU call: prop-wave k_step_h -- bits vs the previous build, then the A/B timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/env_digest.py tools/_build/ref_head.so uav_reinforcement_learning_control_amd/_lib/libquadenv.so > gpurun_out/r4pw_digest.txt 2>&1
echo "digest rc=$?"; tail -3 gpurun_out/r4pw_digest.txt
timeout -k 10 600 python -u tools/step_env_ab.py 65536,4096 3 two=in-tree@QUADENV_PROPW=0 pw2=in-tree pw1=tools/_build/var_pw1.so pw3=tools/_build/var_pw3.so > gpurun_out/r4pw_ab.txt 2>&1
echo "ab rc=$?"; cat gpurun_out/r4pw_ab.txt
