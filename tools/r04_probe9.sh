#!/bin/bash
# round-4 probe: the fp64 IHO mirror's band reads as one stream read 2 / 4 reads ahead (QCART_MIRPIPE 1 / 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
for lib in libqcart_mp2.so libqcart_mp4.so; do
  QCART_LIB=$PWD/$P/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
      -k "iho or table_placements or two_slot or mkl" > gpurun_out/p9_tests_$lib.log 2>&1; rc=$?
  echo "$lib tests rc=$rc $(tail -1 gpurun_out/p9_tests_$lib.log)"; grep FAILED gpurun_out/p9_tests_$lib.log; [ $rc -le 1 ] || exit $rc
done
bash tools/ab_cfg.sh metric 65536 3 libqcart.so libqcart_mp2.so libqcart_mp4.so || exit $?
bash tools/ab_cfg.sh C2 4096 2 libqcart.so libqcart_mp2.so libqcart_mp4.so
