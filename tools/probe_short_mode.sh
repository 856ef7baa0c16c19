#!/bin/bash
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/short
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for n in 180 511; do
  for m in 1 0; do
    QCART_SHORT_MODE0=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/n${n}_m${m} -o run -- python3 $R/tools/short_call_probe.py --variant dev --batch 16 --calls 500 --n-max $n > $OUT/n${n}_m${m}.log 2>&1 || exit 1
    tail -1 $OUT/n${n}_m${m}.log
  done
done
