# round-4 GPU call: the two-rank data-parallel update vs its one-process replay
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_learner.py -k "two_ranks or precomputed or epoch_adv" > gpurun_out/r4_dp_emu.log 2>&1
rc=$?; tail -15 gpurun_out/r4_dp_emu.log; exit $rc
