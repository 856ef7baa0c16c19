#!/bin/bash
# GPU box: the -m gpu suite, the default bench line and the two-rank launcher rehearsal on one device
# (QCART_BENCH_SHARE_DEVICE=1) at the metric's per-rank batch. Usage: bash tools/gpu_suite.sh <tag>
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && tail -3 $OUT/pytest_gpu.log \
 && timeout -k 10 300 python bench.py > $OUT/bench_line.json 2> $OUT/bench.err \
 && cat $OUT/bench_line.json \
 && QCART_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --launch-timeout 360 \
      > $OUT/bench_share2.json 2> $OUT/bench_share2.err \
 && cat $OUT/bench_share2.json
