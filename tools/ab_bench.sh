#!/bin/bash
# A/B the default build against an alternative in-tree library (QCART_LIB) in one GPU call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in "$@"; do
  for rep in 1 2; do
    QCART_LIB="$PWD/deepreinforcementlearningcontrolofquantumcartpoles_amd/$lib" timeout -k 10 300 \
      python bench.py --steps 5 --warmup 1 --no-cpu-baseline > "gpurun_out/ab_${lib}_$rep.log" 2>&1; rc=$?
    echo "$lib rep$rep rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${lib}_$rep.log').read().strip().splitlines()[-1]); print('%.4g env-steps/s  kernel %.2f ms' % (d['value'], d['roofline']['kernel_ms']))" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
