#!/bin/bash
# round-4 probe: the grid R = 17 MODE 0 NaN against the noise-refill variants (all built with the grid TU's own
# -ffp-contract=fast), then the GPU suite, A/Bs and C4 traffic for the shipped candidate (constants by VGPR asm)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
for lib in libqcart_base.so libqcart_nzl.so libqcart_kc0.so libqcart_kcs.so libqcart.so; do
  QCART_LIB=$PWD/$P/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "table_placements" > gpurun_out/p6_tp_$lib.log 2>&1; rc=$?
  echo "$lib table_placements rc=$rc $(tail -1 gpurun_out/p6_tp_$lib.log)"
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p6.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_p6.log; grep FAILED gpurun_out/pytest_p6.log | head; [ $rc -le 1 ] || exit $rc
bash tools/ab_cfg.sh C4 8192 2 libqcart_base.so libqcart.so || exit $?
bash tools/ab_cfg.sh metric 65536 2 libqcart_base.so libqcart.so || exit $?
bash tools/gpu_profile.sh r04k_C4 --config C4 --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p6_prof_C4.txt 2>&1; rc=$?
echo "C4 profile rc=$rc"; exit $rc
