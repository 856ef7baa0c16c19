#!/bin/bash
# round-4 probe: C3 with the backward scan's first composite level read ahead of the backward pass (QCART_PFB 1;
# 2: the second level's reads before the first level's multiply-adds too) — parity against the oracle, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
for lib in libqcart_pfb.so libqcart_pfb2.so; do
  QCART_LIB=$PWD/$P/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 \
      --timeout-method thread -k "qo1025" > gpurun_out/p8_tests_$lib.log 2>&1; rc=$?
  echo "$lib tests rc=$rc $(tail -1 gpurun_out/p8_tests_$lib.log)"; grep FAILED gpurun_out/p8_tests_$lib.log; [ $rc -le 1 ] || exit $rc
done
bash tools/ab_cfg.sh C3 16384 2 libqcart.so libqcart_pfb.so libqcart_pfb2.so
