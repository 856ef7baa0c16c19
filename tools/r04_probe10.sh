#!/bin/bash
# round-4 probe: the fp32 IHO mirror's band reads as one stream read 4 / 8 reads ahead (QCART_MIRPIPE_F32 2 / 3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
for lib in libqcart_f4.so libqcart_f8.so; do
  QCART_LIB=$PWD/$P/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
      -k "fp32 or f32 or iho2048" > gpurun_out/p10_tests_$lib.log 2>&1; rc=$?
  echo "$lib tests rc=$rc $(tail -1 gpurun_out/p10_tests_$lib.log)"; grep FAILED gpurun_out/p10_tests_$lib.log; [ $rc -le 1 ] || exit $rc
done
bash tools/ab_cfg.sh C5 32768 2 libqcart.so libqcart_f4.so libqcart_f8.so
