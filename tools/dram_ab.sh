# A/B tool (not product): the large-batch step forms at the DRAM-bound sizes, in-tree library vs a
# variant build, alternating processes (the same form measured 244 and 290 us at 4M envs in two
# processes of one box: the A/B needs repetitions). usage: bash tools/dram_ab.sh variant.so sizes lanes reps
set -u
V=${1:-tools/_build/var_w6.so}; SIZES=${2:-4194304}; LANES=${3:-1,2}; REPS=${4:-3}
for r in $(seq 1 "$REPS"); do
  timeout -k 10 120 python -u tools/dram_sweep.py "$SIZES" "$LANES" || exit $?
  QUADENV_LIB=$V timeout -k 10 120 python -u tools/dram_sweep.py "$SIZES" "$LANES" || exit $?
done
