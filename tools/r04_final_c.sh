#!/bin/bash
# round-4 final passes on the final library: GPU suite, run table (kernel stats, traffic, bench lines with the CPU
# baseline), SQ instruction-mix passes, then the default bench line (python bench.py, as the driver runs it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/r04_final_a.sh || exit $?
bash tools/sq_configs.sh r04 C5 C3 C4 metric || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "default bench rc=$rc"; grep '^{' gpurun_out/bench_default.log | tail -1; exit $rc
