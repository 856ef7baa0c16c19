#!/bin/bash
# SQ issue/stall counters for the step kernel (separate PMC passes; no trace domains combined).
# usage: tools/gpu_counters.sh TAG [CONFIG] [extra bench.py args, e.g. --batch 32768]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
CONFIG="${2:-metric}"   # bench.py --config
shift; shift || true
EXTRA="$*"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-include-regex k_step --output-format csv \
     -d "$ROOT/gpurun_out/prof_${name}_$TAG" -o run \
     -- python3 "$ROOT/bench.py" --config "$CONFIG" --steps 2 --warmup 1 --no-cpu-baseline $EXTRA > "$ROOT/gpurun_out/prof_${name}_$TAG.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU && \
run sqb SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE && \
run sqc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_COUNT && \
run sqd SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_WR SQ_INSTS_FLAT
[ $? -eq 0 ] && run sqe SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_INST_CYCLES_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS_LOAD
