#!/bin/bash
# GPU box: the -m gpu suite, then C5's cost split — phase stamps (libqcart_stamps.so, fp32 TU) of the R = 16 and
# R = 32 fp32 IHO kernels and the SQ instruction mix of the R = 16 one (tools/sq_configs.sh).
# usage: bash tools/gpu_c5probe.sh TAG
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PKG=deepreinforcementlearningcontrolofquantumcartpoles_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && tail -2 $OUT/pytest_gpu.log \
 && QCART_LIB=$PWD/$PKG/libqcart_stamps.so timeout -k 10 300 python tools/diag_stamps.py C5r16 32768 > $OUT/stamps_C5r16.txt 2>&1 \
 && QCART_LIB=$PWD/$PKG/libqcart_stamps.so timeout -k 10 300 python tools/diag_stamps.py C5 32768 > $OUT/stamps_C5.txt 2>&1 \
 && cat $OUT/stamps_C5r16.txt $OUT/stamps_C5.txt \
 && bash tools/sq_configs.sh $TAG C5r16
