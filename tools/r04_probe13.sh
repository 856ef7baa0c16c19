#!/bin/bash
# round-4 probe: the 'xp' actor loop (tools/bench_loop.py) on the round-3 library against the final one, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
for rep in 1 2; do
  for lib in libqcart_r03.so libqcart.so; do
    QCART_LIB=$PWD/$P/$lib timeout -k 10 300 python tools/bench_loop.py --batch 65536 --steps 20 > gpurun_out/loop_${lib}_$rep.log 2>&1; rc=$?
    echo "$lib rep$rep rc=$rc $(python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/loop_${lib}_$rep.log') if l.startswith('{')][-1]); print('%.2f ms/control step, actor %.2f, replay %.2f' % (d['ms_per_control_step'], d['actor_ms_per_control_step'], d['replay_ms_per_control_step']))" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
