#!/bin/bash
# round-4 probe: a third LDS base (+128 KiB) for the table images past 128 KiB (C5, C4, C3): tests, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
QCART_LIB=$PWD/$P/libqcart_t2g.so timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 \
    --timeout-method thread > gpurun_out/p11_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/p11_tests.log)"; grep FAILED gpurun_out/p11_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/ab_cfg.sh C5 32768 2 libqcart.so libqcart_t2g.so || exit $?
bash tools/ab_cfg.sh C4 8192 2 libqcart.so libqcart_t2g.so || exit $?
bash tools/ab_cfg.sh C3 16384 1 libqcart.so libqcart_t2g.so
