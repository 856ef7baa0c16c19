#!/bin/bash
# round-4 probe: GPU tests on the library with the noise refill's constants defined in place (untied asm) and the
# per-wave LDS noise buffer, same-call A/Bs against the previous library (C4, metric), the C4 traffic passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p5.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_p5.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_cfg.sh C4 8192 3 libqcart_base.so libqcart.so || exit $?
bash tools/ab_cfg.sh metric 65536 2 libqcart_base.so libqcart.so || exit $?
bash tools/ab_cfg.sh C3 16384 1 libqcart_base.so libqcart.so || exit $?
bash tools/gpu_profile.sh r04k_C4 --config C4 --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p5_prof_C4.txt 2>&1; rc=$?
echo "C4 profile rc=$rc"; exit $rc
