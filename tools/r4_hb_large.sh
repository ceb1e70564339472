# round-4 GPU call: k_step_h block size (256 vs 64 envs) at the large batches, state policy by size
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/step_env_ab.py 262144,1048576,2097152,4194304,8388608 2 hb256=in-tree hb64=in-tree@QUADENV_HBLOCK=64 > gpurun_out/r4_hb_large.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_hb_large.txt
