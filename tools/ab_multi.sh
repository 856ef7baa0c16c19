#!/bin/bash
# A/B/C... of in-tree library builds on bench configs, interleaved and repeated, in one GPU call:
#   REPS=2 bash tools/ab_multi.sh "<lib1> <lib2> ..." <cfg>[:batch] ...
# prints "<cfg> <lib> kernel_ms" per run
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
LIBS="$1"; shift
mkdir -p gpurun_out
for rep in $(seq 1 "${REPS:-2}"); do
  for spec in "$@"; do
    c=${spec%%:*}; b=""; [ "$spec" != "$c" ] && b="--batch ${spec##*:}"
    for lib in $LIBS; do
      QCART_LIB="$ROOT/$lib" timeout -k 10 200 python bench.py --config "$c" $b --steps 4 --warmup 1 --no-cpu-baseline \
          > gpurun_out/abm.log 2>&1 || { echo "fail $c $lib"; exit 1; }
      echo "$c $(basename "$lib") $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abm.log | grep -o '[0-9.]*$')"
    done
  done
done
