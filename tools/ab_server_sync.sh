#!/bin/bash
# the server's tick completion by polling an event (default) vs a blocking wait (QCART_SERVER_SYNC=block), at 40 and
# 16 actor processes, n_max = 180, alternating
set -o pipefail
OUT=gpurun_out/ssync
mkdir -p $OUT
for P in 40 16; do
  for s in spin block block spin; do
    if [ $s = block ]; then export QCART_SERVER_SYNC=block; else unset QCART_SERVER_SYNC; fi
    timeout -k 10 200 python tools/bench_dropin.py --procs $P --n-max 180 --kinds server --seconds 4 \
        --out $OUT/p${P}_${s}_$RANDOM.json > $OUT/last.log 2>&1 || exit 1
    echo "P $P $s $(grep -o '"step_calls_per_s": [0-9.e+]*' $OUT/last.log | head -1)"
  done
done
unset QCART_SERVER_SYNC
