#!/bin/bash
# round-4 final pass A: the whole GPU test suite, then the run table (per config: rocprofv3 kernel stats +
# FETCH_SIZE / WRITE_SIZE passes + one bench line with the CPU baseline). Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
TAG=r04 bash tools/run_table.sh
