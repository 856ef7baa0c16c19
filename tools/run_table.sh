#!/bin/bash
# BASELINE.md §4 run table: for each config, rocprofv3 kernel stats + FETCH/WRITE PMC passes
# (tools/gpu_profile.sh, tag ${TAG:-r02}_<cfg>) and one bench line with the CPU baseline. Per-GPU batches:
# C4 65 536 / 8 GPUs, C5 262 144 / 8 GPUs. Stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
for spec in "C1:1" "C2:4096" "C3:16384" "C4:8192" "C5:32768" "metric:65536"; do
  cfgname=${spec%%:*}; b=${spec##*:}
  bash tools/gpu_profile.sh "${TAG:-r02}_$cfgname" --config "$cfgname" --batch "$b" --steps 3 --warmup 1 --no-cpu-baseline \
      > "gpurun_out/rt_prof_$cfgname.txt" 2>&1; rc=$?
  echo "$cfgname profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$ROOT"
  timeout -k 10 300 python bench.py --config "$cfgname" --batch "$b" --steps 3 --warmup 1 --cpu-seconds 6 \
      > "gpurun_out/rt_$cfgname.log" 2>&1; rc=$?
  echo "$cfgname bench rc=$rc $(grep -o '"value": [0-9.e+]*' gpurun_out/rt_$cfgname.log | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
