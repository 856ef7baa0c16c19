#!/bin/bash
# End-of-round passes on the final library, one GPU call: the GPU test suite, the run table (per config:
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes + one bench line with the CPU baseline), the SQ
# instruction-mix passes of the batched configs' step kernels, then the default bench line (python bench.py, as
# the driver runs it). Stops at the first failing step.  usage: bash tools/final_passes.sh <tag>
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/run_table.sh || exit $?
bash tools/sq_configs.sh "$TAG" C5 C3 C4 metric || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "default bench rc=$rc"; grep '^{' gpurun_out/bench_default.log | tail -1; exit $rc
