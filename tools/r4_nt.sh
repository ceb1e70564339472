# round-4 GPU call: nt cache policy on the env-state tile loads / stores (A/B builds) at 4M, 1M, 65,536 envs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/step_env_ab.py 4194304,1048576,65536 2 base=in-tree ldnt=tools/_build/var_ldnt.so stnt=tools/_build/var_stnt.so bnt=tools/_build/var_bnt.so > gpurun_out/r4_nt.txt 2>&1
echo "rc=$?"; cat gpurun_out/r4_nt.txt
