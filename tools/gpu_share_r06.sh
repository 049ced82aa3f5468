#!/bin/bash
# Exact-path work sharing (libavz_dev.so): IBM exact + parity GPU tests, then a same-box A/B
# against the shipped library.
set -o pipefail
out=gpurun_out/r06sh
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
AVZ_LIB=$D/libavz_dev.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ibm_exact.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
bash tools/gpu_ab_r06.sh r06sh/ab 2 \
  "base|AVZ_LIB=$D/libavz.so python bench.py --no-cpu --no-secondary --steps 20" \
  "share|AVZ_LIB=$D/libavz_dev.so python bench.py --no-cpu --no-secondary --steps 20"
