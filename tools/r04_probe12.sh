#!/bin/bash
# round-4 end-to-end refresh on the final library: the actor loop with 'xp' input and with the measurement record
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_loop.py --batch 65536 --steps 20 > gpurun_out/loop_xp.log 2>&1; rc=$?
echo "xp rc=$rc"; grep '^{' gpurun_out/loop_xp.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_loop.py --batch 65536 --steps 10 --input measurements > gpurun_out/loop_meas.log 2>&1; rc=$?
echo "measurements rc=$rc"; grep '^{' gpurun_out/loop_meas.log | tail -1; exit $rc
