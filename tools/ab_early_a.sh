#!/bin/bash
# A/B of the early activation loads (HEAD default) against the late form (exp/base5.so = NERF_X6W_LATE_A-equivalent
# build of the previous HEAD): three alternating C2 rounds.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
VARIANTS="base5 head" ROUNDS=${ROUNDS:-3} tools/ab_x6.sh
