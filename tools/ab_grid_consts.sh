#!/bin/bash
# A/B (alternating, one call): the grid kernels with host-folded step constants (gh) and + per-step kernarg re-read
# (gkh) against the shipped library, at C3 and C4
set -o pipefail
P=deepreinforcementlearningcontrolofquantumcartpoles_amd
bash tools/ab_alt.sh $P/libqcart.so $P/libqcart_gkh.so C3:16384 C4:8192 && \
bash tools/ab_alt.sh $P/libqcart.so $P/libqcart_gh.so C3:16384 C4:8192
