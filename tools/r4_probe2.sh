# round-4 GPU call: the launch floor at the step kernel's shapes; the learner round's phases with the barrier waits split out
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/_build/launch_floor > gpurun_out/r4_launch_floor.txt 2>&1
echo "floor rc=$?"; cat gpurun_out/r4_launch_floor.txt
timeout -k 10 300 python -u tools/probe/probe_learner.py > gpurun_out/r4_probe_learner.txt 2>&1
echo "probe rc=$?"; cat gpurun_out/r4_probe_learner.txt
