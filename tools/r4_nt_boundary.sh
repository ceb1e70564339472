# round-4 GPU call: k_step_h with the state cache policy pinned (QUADENV_NT=0 / 1) around the
# policy's boundaries (65,536 .. 196,608 and 1M .. 2M envs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/step_env_ab.py 65536,98304,131072,196608,1572864 2 nt0=in-tree@QUADENV_NT=0 nt1=in-tree@QUADENV_NT=1 > gpurun_out/r4_nt_boundary.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_nt_boundary.txt
