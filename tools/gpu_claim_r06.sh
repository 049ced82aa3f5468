#!/bin/bash
# Blind first claim + exact-table prefetch (libavz_dev.so) against the same split build of HEAD
# (libavz_devbase.so): exact + parity GPU tests, then a same-box A/B.
set -o pipefail
out=gpurun_out/${TAG:-r06cl}
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
AVZ_LIB=$D/libavz_dev.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ibm_exact.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/gpu_ab_r06.sh ${TAG:-r06cl}/ab 3 \
  "devbase|AVZ_LIB=$D/libavz_devbase.so python bench.py --no-cpu --no-secondary --steps 20" \
  "claim|AVZ_LIB=$D/libavz_dev.so python bench.py --no-cpu --no-secondary --steps 20"
