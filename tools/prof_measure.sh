#!/bin/bash
# rocprofv3 kernel statistics of tools/bench_measure.py -> gpurun_out/prof_measure_<tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_${BENCH:-bench_measure}_$TAG" -o run \
    -- python3 "$ROOT/tools/${BENCH:-bench_measure}.py" ${BARGS:-} > "$ROOT/gpurun_out/prof_${BENCH:-bench_measure}_$TAG.log" 2>&1; rc=$?
echo "rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/prof_${BENCH:-bench_measure}_$TAG.log" | tail -1
cut -d, -f1-8 "$ROOT/gpurun_out/prof_${BENCH:-bench_measure}_$TAG/run_kernel_stats.csv"
exit $rc
