# round-4 GPU call: k_step_h with a waves-per-EU floor of 7 (QD_H_WAVES=7: 72 VGPRs, 5 spilled) vs the
# default build at the DRAM sizes (64-env blocks, nt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/step_env_ab.py 1048576,3145728,8388608 2 base=in-tree hw7=tools/_build/var_hw7.so > gpurun_out/r4_hw2.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_hw2.txt
