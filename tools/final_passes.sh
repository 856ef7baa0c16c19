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
bash tools/sq_configs.sh "$TAG" C5 C3 C4 metric C2 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "default bench rc=$rc"; grep '^{' gpurun_out/bench_default.log | tail -1; [ $rc -eq 0 ] || exit $rc
# the end-to-end actor loop (both reset modes) and the drop-in under the reference's process model
for rs in deferred immediate; do
  timeout -k 10 300 python tools/bench_loop.py --batch 65536 --steps 10 --input xp --reset $rs > gpurun_out/${TAG}_loop_$rs.log 2>&1 || exit $?
  echo "loop $rs $(grep -o '"ms_per_control_step": [0-9.]*' gpurun_out/${TAG}_loop_$rs.log)"
done
timeout -k 10 600 python tools/bench_dropin.py --procs 1,8,16 --kinds server,gpu,cpu --seconds 4 --n-max 511 \
    --out gpurun_out/${TAG}_dropin_procs_511.json > gpurun_out/${TAG}_dropin_procs_511.log 2>&1 || exit $?
grep '^{' gpurun_out/${TAG}_dropin_procs_511.log | cut -c1-120
