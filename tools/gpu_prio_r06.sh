#!/bin/bash
# Same-box A/B: wave priority of the analysis loop over the exact phase (-DAVZ_XPRIO=2) against
# the same split development build without it.
set -o pipefail
D=real-time-audio-visual-zooming_amd/avz
bash tools/gpu_ab_r06.sh ${TAG:-r06prio}/ab 3 \
  "dev|AVZ_LIB=$D/libavz_dev.so python bench.py --no-cpu --no-secondary --steps 20" \
  "prio2|AVZ_LIB=$D/libavz_p2.so python bench.py --no-cpu --no-secondary --steps 20"
