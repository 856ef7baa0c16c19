#!/bin/bash
# mactor parity tests, then bench_mactor for the default build and each alternative library given.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mactor.py tests/test_gpu_actor.py > gpurun_out/ma.log 2>&1; rc=$?
tail -2 gpurun_out/ma.log; [ $rc -eq 0 ] || exit $rc
for lib in libqcart.so "$@"; do
  for ch in 1024 2048; do
    QCART_LIB="$PWD/deepreinforcementlearningcontrolofquantumcartpoles_amd/$lib" timeout -k 10 120 \
      python tools/bench_mactor.py --chunk $ch > gpurun_out/bma_${lib}_$ch.log 2>&1; rc=$?
    echo "$lib chunk $ch rc=$rc $(grep -o '"ms_per_call": [0-9.]*' gpurun_out/bma_${lib}_$ch.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
