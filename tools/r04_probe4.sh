#!/bin/bash
# round-4 probe: which noise-refill variant breaks the grid R = 17 MODE 0 kernel (table-placement test per
# library), then same-call A/Bs (C4, metric), the fixed per-launch cost, the C4 traffic and the drop-in sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
for lib in libqcart.so libqcart_gsc0.so libqcart_gkc0.so libqcart_glib0.so; do
  QCART_LIB=$PWD/$P/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "table_placements" > gpurun_out/p4_tp_$lib.log 2>&1; rc=$?
  echo "$lib table_placements rc=$rc $(tail -1 gpurun_out/p4_tp_$lib.log)"
  [ $rc -le 1 ] || exit $rc
done
bash tools/ab_cfg.sh C4 8192 2 libqcart_base.so libqcart_kc.so libqcart.so libqcart_gsc0.so || exit $?
bash tools/ab_cfg.sh metric 65536 2 libqcart_base.so libqcart_kc.so libqcart.so || exit $?
timeout -k 10 180 python tools/diag_overhead.py > gpurun_out/p4_overhead.log 2>&1; echo "overhead rc=$?"; grep k_step gpurun_out/p4_overhead.log
bash tools/gpu_profile.sh r04k_C4 --config C4 --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p4_prof_C4.txt 2>&1; rc=$?
echo "C4 profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/r04_dropin_env.sh
