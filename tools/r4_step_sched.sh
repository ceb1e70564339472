# round-4 GPU call: the env kernels built with the backend's alternative scheduling strategies
# (max-ilp / max-memory-clause) vs the default build -- step digests and per-launch times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/step_env_ab.py 4096,65536,1048576 5 ilp=tools/_build/var_ilp.so base=in-tree > gpurun_out/r4_step_sched2.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_step_sched2.txt
