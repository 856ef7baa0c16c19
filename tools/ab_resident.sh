#!/bin/bash
# the step server's resident kernel: its GPU tests, then step calls/s at the IHO driver's n_max = 180 with the
# resident path against the ticks (QCART_SERVER_RESIDENT=0), alternating, at P = 16 and the drivers' 40 actor
# processes, and the oracle processes for reference. Usage: bash tools/ab_resident.sh [tag]
set -o pipefail
OUT=gpurun_out/${1:-resident}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py tests/test_server_protocol.py -x -v --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for P in 16 40; do
  for s in res tick tick res; do
    if [ $s = res ]; then unset QCART_SERVER_RESIDENT; else export QCART_SERVER_RESIDENT=0; fi
    timeout -k 10 200 python tools/bench_dropin.py --procs $P --n-max 180 --kinds server --seconds 4 \
        --out $OUT/p${P}_${s}_$RANDOM.json > $OUT/last.log 2>&1 || { tail -20 $OUT/last.log; exit 1; }
    echo "P $P $s $(grep -o '"step_calls_per_s": [0-9.e+]*' $OUT/last.log | head -1)"
  done
done
unset QCART_SERVER_RESIDENT
for P in 16 40; do
  timeout -k 10 200 python tools/bench_dropin.py --procs $P --n-max 180 --kinds cpu --seconds 4 \
      --out $OUT/p${P}_cpu.json > $OUT/cpu.log 2>&1 && echo "P $P cpu $(grep -o '"step_calls_per_s": [0-9.e+]*' $OUT/cpu.log | head -1)"
done
