#!/bin/bash
# the grid drivers' process model through the step server against the oracle processes: QO (x_n = 171) and IQO
# (x_n = 521) at their driver defaults, 16 and 40 actor processes, with the driver's get_moments per control interval.
# Usage: bash tools/ab_grid_dropin.sh [tag]
set -o pipefail
OUT=gpurun_out/${1:-grid_dropin}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for fam in inverted_quartic quartic; do
  timeout -k 10 400 python tools/bench_dropin.py --family $fam --procs 16,40 --kinds server,cpu --seconds 4 --driver-loop \
      --out $OUT/$fam.json > $OUT/$fam.log 2>&1 || { tail -20 $OUT/$fam.log; exit 1; }
  grep '^{' $OUT/$fam.log | cut -c1-110
done
