#!/bin/bash
# SQ stall-breakdown counters for the step kernel (one PMC pass; no trace domains combined).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
   --output-format csv -d "$ROOT/gpurun_out/prof_sq_$TAG" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_sq_$TAG.log" 2>&1; rc=$?
echo "sq rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE \
   --output-format csv -d "$ROOT/gpurun_out/prof_sq2_$TAG" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_sq2_$TAG.log" 2>&1; rc=$?
echo "sq2 rc=$rc"
exit $rc
