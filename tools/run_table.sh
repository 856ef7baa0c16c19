#!/bin/bash
# BASELINE.md §4 run table: for each config, rocprofv3 kernel stats + FETCH/WRITE PMC passes
# (tools/gpu_profile.sh, tag ${TAG:-r02}_<cfg>) and one bench line with the CPU baseline. Per-GPU batches:
# C4 65 536 / 8 GPUs, C5 262 144 / 8 GPUs. Stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
# config:batch:steps:warmup — the short launches (C1 0.2 ms, C2 1.6 ms) get 30 warm-up launches, so that every config is
# timed on a GPU that has run for at least ~50 ms (one warm-up launch of C2 left the clock ramping: 1.61 ms per launch
# after 1 warm-up vs 1.54 after 30 in one call, profiles/r05_c2_warmup.txt)
for spec in "C1:1:30:30" "C2:4096:30:30" "C3:16384:3:1" "C4:8192:3:1" "C5:32768:3:1" "metric:65536:3:1"; do
  IFS=: read -r cfgname b st wu <<< "$spec"
  bash tools/gpu_profile.sh "${TAG:-r02}_$cfgname" --config "$cfgname" --batch "$b" --steps "$st" --warmup "$wu" --no-cpu-baseline \
      > "gpurun_out/rt_prof_$cfgname.txt" 2>&1; rc=$?
  echo "$cfgname profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$ROOT"
  timeout -k 10 300 python bench.py --config "$cfgname" --batch "$b" --steps "$st" --warmup "$wu" --cpu-seconds 6 \
      > "gpurun_out/rt_$cfgname.log" 2>&1; rc=$?
  echo "$cfgname bench rc=$rc $(grep -o '"value": [0-9.e+]*' gpurun_out/rt_$cfgname.log | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
