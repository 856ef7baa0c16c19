#!/bin/bash
# round-4 final pass B: SQ instruction-mix passes of the four batched configs' step kernels, and the drop-in under
# the reference's process model at the metric's N = 512
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/sq_configs.sh r04 C5 C3 C4 metric || exit $?
timeout -k 10 400 python tools/bench_dropin.py --procs 1,8,16 --seconds 5 --kinds gpu,cpu --n-max 511 \
    --out gpurun_out/dropin_procs_511.json > gpurun_out/dropin_procs_511.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/dropin_procs_511.log
exit $rc
