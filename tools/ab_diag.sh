#!/bin/bash
# A/B k_step launch time (tools/diag_actions.py, random actions) of in-tree libraries, alternating,
# in one GPU call: bash tools/ab_diag.sh libqcart.so libqcart_prev.so [extra diag args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; B=$2; shift 2
P=$PWD/deepreinforcementlearningcontrolofquantumcartpoles_amd
for r in 1 2; do
  for l in $A $B; do
    QCART_LIB=$P/$l timeout -k 10 200 python tools/diag_actions.py --only random "$@" 2>&1 | grep -v amdgpu.ids | sed "s/^/$l /" || exit 1
  done
done
