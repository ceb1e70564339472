# round-4 GPU call: k_step_hd with the LEAN helper image (reset obs formed by the step lane) -- its
# parity tests, then the A/B against the full image (QD_HD_LEAN=0 build) at 4M / 8M envs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "0d or four_million or form_selection" --timeout 240 --timeout-method thread > gpurun_out/r4_lean_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_lean_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/step_env_ab.py 4194304,8388608 3 lean=in-tree full=tools/_build/var_hdfat.so > gpurun_out/r4_lean_ab.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_lean_ab.txt
