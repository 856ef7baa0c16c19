#!/bin/bash
# Quick GPU pass for kernel iterations: parity tests then the action-layout timing diagnostic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 600 "$@" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/diag_actions.py > gpurun_out/diag.log 2>&1; rc2=$?
grep -v amdgpu.ids gpurun_out/diag.log
exit $(( rc != 0 ? rc : rc2 ))
