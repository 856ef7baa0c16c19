#!/bin/bash
# round-4 probe: GPU tests on the rebuilt library (noise refill constants in place), same-call A/B of the
# previous library against it (C4, metric, C3), the C4 traffic passes, and the drop-in queue-setting sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p3.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_p3.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_cfg.sh C4 8192 3 libqcart_base.so libqcart_kc.so libqcart.so || exit $?
bash tools/ab_cfg.sh metric 65536 2 libqcart_base.so libqcart_kc.so libqcart.so || exit $?
bash tools/ab_cfg.sh C3 16384 1 libqcart_base.so libqcart_kc.so libqcart.so || exit $?
bash tools/gpu_profile.sh r04k_C4 --config C4 --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p3_prof_C4.txt 2>&1; rc=$?
echo "C4 profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python tools/diag_overhead.py > gpurun_out/p3_overhead.log 2>&1; echo "overhead rc=$?"; grep k_step gpurun_out/p3_overhead.log
bash tools/r04_dropin_env.sh
