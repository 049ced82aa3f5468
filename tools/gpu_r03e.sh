#!/bin/bash
# stamps of waves 1 and 3, then bench A/B of the default vs the L2-prefetch build
set -o pipefail
bash tools/stamps.sh ${1}_st 1 3 || exit 1
REPS=3 BENCH_ARGS=--no-secondary bash tools/ab_libs.sh ${1}_pf libavz.so libavz_pf.so
