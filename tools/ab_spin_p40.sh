#!/bin/bash
# step-server client poll window with 40 actor processes on the box's 16-CPU share (n_max = 180): default (20 us when
# the clients outnumber the CPUs) vs 0 / 5 / 50 us, alternating
set -o pipefail
OUT=gpurun_out/spin40
mkdir -p $OUT
for rep in 1 2; do
  for s in default 0 5 50; do
    if [ $s = default ]; then unset QCC_SPIN_US; else export QCC_SPIN_US=$s; fi
    timeout -k 10 200 python tools/bench_dropin.py --procs 40 --n-max 180 --kinds server --seconds 4 \
        --out $OUT/spin_${s}_$rep.json > /dev/null 2>&1 || exit 1
    echo "spin $s rep $rep $(grep -o '"step_calls_per_s": [0-9.e+]*' $OUT/spin_${s}_$rep.json | head -1)"
  done
done
unset QCC_SPIN_US
