#!/bin/bash
# Profiling tool (not product): the first timed region of a fresh process (what the driver's one
# bench run sees) under variants: as bench.py, + the timed graph replayed once more (WARM_G), + a
# spin kernel before the region (SPIN_CYCLES), + the region's host path run once with no launches
# (DRY) or around the warm-up graph (DRYG). Three fresh processes per variant.
set -u
cd "$(dirname "$0")/../.."
VARIANTS=${VARIANTS:-"base WARM_G=1 SPIN_CYCLES=2000000 SPIN_CYCLES=20000000"}
for rep in 1 2 3; do
  for v in $VARIANTS; do
    echo "--- $v"
    if [ "$v" = base ]; then timeout -k 10 120 python tools/probe/wall_overhead.py auto 65536 20 8 || exit $?
    else env $v timeout -k 10 120 python tools/probe/wall_overhead.py auto 65536 20 8 || exit $?; fi
  done
done
