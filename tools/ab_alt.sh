#!/bin/bash
# A/B of two in-tree library builds (QCART_LIB) in alternating order (A B B A per config), one GPU call:
#   bash tools/ab_alt.sh <libA> <libB> <cfg>[:batch] ...     (cfg "metric" = the default bench workload)
# kernel_ms per run -> gpurun_out/abalt_<cfg>_<tag><rep>.log
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
A="$1"; B="$2"; shift 2
mkdir -p gpurun_out
for spec in "$@"; do
  c=${spec%%:*}; b=""; [ "$spec" != "$c" ] && b="--batch ${spec##*:}"
  cf="--config $c"; [ "$c" = metric ] && cf=""
  rep=0
  for tag in A B B A; do
    rep=$((rep + 1))
    lib=$A; [ $tag = B ] && lib=$B
    QCART_LIB="$ROOT/$lib" timeout -k 10 240 python bench.py $cf $b --steps 4 --warmup 1 --no-cpu-baseline \
        > "gpurun_out/abalt_${c}_$tag$rep.log" 2>&1 || { echo "fail $c $tag"; exit 1; }
    echo "$c $tag $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abalt_${c}_$tag$rep.log)"
  done
done
