# round-4 GPU call: the persistent, prefetching lane-group step (k_step_gp) vs k_step_g at the DRAM sizes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/step_env_ab.py 4194304,1048576 2 g1=in-tree@QUADENV_LANES=1 g2=in-tree@QUADENV_LANES=2 p512=in-tree@QUADENV_LANES=2,QUADENV_PERSIST=512 p768=in-tree@QUADENV_LANES=2,QUADENV_PERSIST=768 p1024=in-tree@QUADENV_LANES=2,QUADENV_PERSIST=1024 p2048=in-tree@QUADENV_LANES=2,QUADENV_PERSIST=2048 > gpurun_out/r4_persist.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_persist.txt
