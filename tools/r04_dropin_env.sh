#!/bin/bash
# Drop-in under the reference's process model (P actor processes sharing one GPU) with the HIP runtime's queue
# settings varied: default, one hardware queue per process, copies as blit kernels instead of SDMA, and both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-511}
for setting in default hwq1 nosdma hwq1_nosdma; do
    case $setting in
        default) envs=() ;;
        hwq1) envs=(GPU_MAX_HW_QUEUES=1) ;;
        nosdma) envs=(HSA_ENABLE_SDMA=0) ;;
        hwq1_nosdma) envs=(GPU_MAX_HW_QUEUES=1 HSA_ENABLE_SDMA=0) ;;
    esac
    env "${envs[@]}" timeout -k 10 200 python tools/bench_dropin.py --procs 1,8,16 --seconds 3 --kinds gpu \
        --n-max "$N" --out "gpurun_out/dropin_env_${setting}_${N}.json" > "gpurun_out/dropin_env_${setting}_${N}.log" 2>&1
    rc=$?
    echo "$setting rc=$rc"
    grep '^{' "gpurun_out/dropin_env_${setting}_${N}.log"
    [ $rc -eq 0 ] || exit $rc
done
