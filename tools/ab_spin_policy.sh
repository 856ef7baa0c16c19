#!/bin/bash
# the new client poll policy (no poll once the clients outnumber the usable CPUs) against round 5's 20 us, alternating,
# at the drivers' 32 / 40 actor processes; then the 40-process oracle for reference (n_max = 180)
set -o pipefail
OUT=gpurun_out/spinpol
mkdir -p $OUT
for P in 32 40; do
  for s in new old old new; do
    if [ $s = new ]; then unset QCC_SPIN_US; else export QCC_SPIN_US=20; fi
    timeout -k 10 200 python tools/bench_dropin.py --procs $P --n-max 180 --kinds server --seconds 4 \
        --out $OUT/p${P}_${s}_$RANDOM.json > $OUT/last.log 2>&1 || exit 1
    echo "P $P $s $(grep -o '"step_calls_per_s": [0-9.e+]*' $OUT/last.log | head -1)"
  done
done
unset QCC_SPIN_US
timeout -k 10 200 python tools/bench_dropin.py --procs 40 --n-max 180 --kinds server,cpu --seconds 4 \
    --out $OUT/p40_final.json > $OUT/final.log 2>&1 && grep '^{' $OUT/final.log | cut -c1-100
