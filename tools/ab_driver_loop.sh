#!/bin/bash
# the IHO driver's per-process loop through the step server (80 steps + x_expectation per control interval) against the
# oracle processes doing the same, at n_max = 180 and the drivers' 16 / 40 actors. Usage: bash tools/ab_driver_loop.sh [tag]
set -o pipefail
OUT=gpurun_out/${1:-driverloop}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for P in 16 40; do
  timeout -k 10 300 python tools/bench_dropin.py --procs $P --n-max 180 --kinds server,cpu --seconds 4 --driver-loop \
      --out $OUT/p${P}.json > $OUT/p${P}.log 2>&1 || { tail -20 $OUT/p${P}.log; exit 1; }
  grep '^{' $OUT/p${P}.log | cut -c1-120
done
