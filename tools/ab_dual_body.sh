#!/bin/bash
# alternating: the metric step body in the DUAL kernel vs the single-slot kernel, on a batch without two-slot blocks
set -o pipefail
for r in 1 2; do
  QCART_DUAL=1 timeout -k 10 200 python tools/probe_dual_body.py || exit 1
  QCART_DUAL=0 timeout -k 10 200 python tools/probe_dual_body.py || exit 1
  QCART_DUAL=0 timeout -k 10 200 python tools/probe_dual_body.py || exit 1
  QCART_DUAL=1 timeout -k 10 200 python tools/probe_dual_body.py || exit 1
done
