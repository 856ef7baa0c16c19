#!/bin/bash
# A/B of environment settings (QCART_DUAL, QCART_TAB_MODE, ...) on bench configs, one GPU call:
#   bash tools/ab_envs.sh "<cfg>[:batch] ..." "A-env" "B-env" [...]     e.g. "metric C2 C4:8192" "QCART_DUAL=0" ""
# Each (config, setting) runs twice, alternating, so box-clock drift shows; kernel_ms -> stdout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
CFGS="$1"; shift
mkdir -p gpurun_out
for spec in $CFGS; do
  c=${spec%%:*}; b=""; [ "$spec" != "$c" ] && b="--batch ${spec##*:}"
  for rep in 1 2; do
    i=0
    for setting in "$@"; do
      i=$((i + 1))
      log="gpurun_out/abe_${c}_${i}_${rep}.log"
      env $setting timeout -k 10 300 python bench.py --config "$c" $b --steps 4 --warmup 1 --no-cpu-baseline > "$log" 2>&1
      rc=$?
      echo "$c [$setting] rep$rep rc=$rc $(grep -o '"kernel_ms": [0-9.]*' "$log")"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
