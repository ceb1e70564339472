# round-4 GPU call: k_step_h with default vs nt tile loads+stores across batch sizes (+ the size-default form)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/step_env_ab.py 4096,32768,262144,524288,2097152 2 \
  h=tools/_build/var_dflt.so@QUADENV_LANES=0 hnt=in-tree@QUADENV_LANES=0 \
  dflt=tools/_build/var_dflt.so@QUADENV_LANES=-1 dfltnt=in-tree@QUADENV_LANES=-1 > gpurun_out/r4_nt_sizes.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_nt_sizes.txt
