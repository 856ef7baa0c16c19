#!/bin/bash
# A/B of two in-tree library builds (QCART_LIB) on bench configs, in one GPU call:
#   bash tools/ab_configs.sh <libA> <libB> <cfg>[:batch] ...
# kernel_ms per config and build -> gpurun_out/ab_<cfg>_<A|B>.log
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
A="$1"; B="$2"; shift 2
mkdir -p gpurun_out
for spec in "$@"; do
  c=${spec%%:*}; b=""; [ "$spec" != "$c" ] && b="--batch ${spec##*:}"
  for tag in A B; do
    lib=$A; [ $tag = B ] && lib=$B
    QCART_LIB="$ROOT/$lib" timeout -k 10 200 python bench.py --config "$c" $b --steps 4 --warmup 1 --no-cpu-baseline \
        > "gpurun_out/ab_${c}_$tag.log" 2>&1 || { echo "fail $c $tag"; exit 1; }
    echo "$c $tag $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_${c}_$tag.log)"
  done
done
