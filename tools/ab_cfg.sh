#!/bin/bash
# A/B in-tree libraries (QCART_LIB) on one run-table config in one GPU call, interleaved:
#   tools/ab_cfg.sh CONFIG BATCH REPS lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=$1; B=$2; REPS=$3; shift 3
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    QCART_LIB="$PWD/deepreinforcementlearningcontrolofquantumcartpoles_amd/$lib" timeout -k 10 300 \
      python bench.py --config "$CFG" --batch "$B" --steps 3 --warmup 1 --no-cpu-baseline > "gpurun_out/ab_${CFG}_${lib}_$rep.log" 2>&1; rc=$?
    echo "$CFG $lib rep$rep rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${CFG}_${lib}_$rep.log').read().strip().splitlines()[-1]); print('%.4g env-steps/s  kernel %.2f ms' % (d['value'], d['roofline']['kernel_ms']))" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
