#!/bin/bash
# the resident kernel with the request's slot image kept in LDS (MODE 2) against the tables read from L2 every request
# (QCART_RESIDENT_MODE=0): one client's latency (C and Python) and step calls/s of 16 / 40 actor processes at n_max = 180,
# alternating. Usage: bash tools/ab_resident_mode.sh [tag]
set -o pipefail
OUT=gpurun_out/${1:-rmode}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in lds l2; do
  if [ $m = l2 ]; then export QCART_RESIDENT_MODE=0; else unset QCART_RESIDENT_MODE; fi
  timeout -k 10 200 python tools/probe_resident_lat.py --calls 20000 > $OUT/lat_$m.jsonl 2> $OUT/lat_$m.err || exit 1
  echo "$m $(head -1 $OUT/lat_$m.jsonl)"
done
for P in 16 40; do
  for m in lds l2 l2 lds; do
    if [ $m = l2 ]; then export QCART_RESIDENT_MODE=0; else unset QCART_RESIDENT_MODE; fi
    timeout -k 10 200 python tools/bench_dropin.py --procs $P --n-max 180 --kinds server --seconds 4 \
        --out $OUT/p${P}_${m}_$RANDOM.json > $OUT/last.log 2>&1 || { tail -20 $OUT/last.log; exit 1; }
    echo "P $P $m $(grep -o '"step_calls_per_s": [0-9.e+]*' $OUT/last.log | head -1)"
  done
done
