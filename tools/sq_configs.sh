#!/bin/bash
# SQ instruction-mix passes (tools/gpu_counters.sh) for the step kernels of the run-table configs:
# usage: tools/sq_configs.sh TAG [cfg ...]   (default: C5 C3 C4 metric; per-GPU batches of the run table)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r04}"; shift || true
CFGS="${*:-C5 C3 C4 metric}"
for c in $CFGS; do
  case $c in C2) b=4096;; C3) b=16384;; C4) b=8192;; C5|C5r16) b=32768;; *) b=65536;; esac
  bash "$ROOT/tools/gpu_counters.sh" "${TAG}_$c" "$c" --batch $b || exit $?
done
