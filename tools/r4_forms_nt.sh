# round-4 GPU call: step forms (k_step_h / k_step_g<1> / k_step_g<2>) x cache policy (default / nt
# loads+stores) at 65,536 .. 8M envs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/step_env_ab.py 4194304,8388608,1048576,65536 2 \
  h=in-tree@QUADENV_LANES=0 hnt=tools/_build/var_bnt.so@QUADENV_LANES=0 \
  g1=in-tree@QUADENV_LANES=1 g1nt=tools/_build/var_bnt.so@QUADENV_LANES=1 \
  g2=in-tree@QUADENV_LANES=2 g2nt=tools/_build/var_bnt.so@QUADENV_LANES=2 > gpurun_out/r4_forms_nt.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_forms_nt.txt
