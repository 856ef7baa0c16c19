#!/bin/bash
# round-4 probe: per-phase stamps of the C5 / C3 / C4 / metric step loops, and the drop-in under the reference's
# process model (P actor processes on one GPU vs P oracle processes on host cores)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
QCART_LIB=$PWD/$P/libqcart_stamps32.so timeout -k 10 120 python tools/diag_stamps.py C5 32768 > gpurun_out/stamps_C5.txt 2>&1 || exit $?
QCART_LIB=$PWD/$P/libqcart_stampsg.so timeout -k 10 120 python tools/diag_stamps.py C3 16384 > gpurun_out/stamps_C3.txt 2>&1 || exit $?
QCART_LIB=$PWD/$P/libqcart_stampsg.so timeout -k 10 120 python tools/diag_stamps.py C4 8192 > gpurun_out/stamps_C4.txt 2>&1 || exit $?
QCART_LIB=$PWD/$P/libqcart_stampsi.so timeout -k 10 120 python tools/diag_stamps.py 511 0 > gpurun_out/stamps_metric.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps_*.txt | head -80
timeout -k 10 400 python tools/bench_dropin.py --procs 1,8,16 --seconds 5 --kinds gpu,cpu --out gpurun_out/dropin_procs.json > gpurun_out/dropin_procs.log 2>&1; rc=$?
cat gpurun_out/dropin_procs.log | grep -v amdgpu.ids
exit $rc
