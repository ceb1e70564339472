# round-4 GPU call: the config-4 shape (8 ranks x 65,536 envs) rehearsed on one GPU over gloo
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/config4_rehearsal.py 8 65536 1024 8 > gpurun_out/r4_config4.txt 2>&1
rc=$?; tail -c 3000 gpurun_out/r4_config4.txt; exit $rc
