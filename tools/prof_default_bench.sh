#!/bin/bash
# rocprofv3 --kernel-trace --stats of the default bench line (python bench.py, exactly as the driver runs it): the
# k_step average it reports must agree with the line's roofline.kernel_ms. usage: bash tools/prof_default_bench.sh TAG
set -o pipefail
TAG=${1:?tag}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_default_$TAG" -o run \
    -- python3 "$ROOT/bench.py" > "$ROOT/gpurun_out/prof_default_$TAG.log" 2>&1 || exit $?
grep '^{' "$ROOT/gpurun_out/prof_default_$TAG.log" | tail -1 | cut -c1-200
grep k_step "$ROOT/gpurun_out/prof_default_$TAG/run_kernel_stats.csv"
