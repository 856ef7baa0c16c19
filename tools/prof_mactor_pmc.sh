#!/bin/bash
# PMC passes (one rocprofv3 run each) over the measurement actor's convolution kernels.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex 'k_mconv|k_mfc' --output-format csv \
     -d "$ROOT/gpurun_out/prof_${name}_$TAG" -o run \
     -- python3 "$ROOT/tools/bench_mactor.py" --batch 8192 --reps 1 ${BARGS:-} > "$ROOT/gpurun_out/prof_${name}_$TAG.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run mca SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD && \
run mcb SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
