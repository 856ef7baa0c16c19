#!/bin/bash
# rocprofv3 passes on the bench workload: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950). Outputs under gpurun_out/prof_*.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
shift || true
BENCH_ARGS="${*:---steps 5 --warmup 1 --no-cpu-baseline}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_kt_$TAG" -o run \
    -- python3 "$ROOT/bench.py" $BENCH_ARGS > "$ROOT/gpurun_out/prof_kt_$TAG.log" 2>&1; rc=$?
echo "kernel-trace rc=$rc"; tail -2 "$ROOT/gpurun_out/prof_kt_$TAG.log"
[ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$ROOT/gpurun_out/prof_pmc_${C}_$TAG" -o run \
      -- python3 "$ROOT/bench.py" $BENCH_ARGS --steps 2 --warmup 1 > "$ROOT/gpurun_out/prof_pmc_${C}_$TAG.log" 2>&1; rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
find "$ROOT/gpurun_out" -name "*.csv" -path "*prof_*$TAG*" | head -20
