#!/bin/bash
# Work sharing for the per-bin kernels (N = 512, IRM): all GPU tests on libavz_dev.so, then a
# same-box A/B of the 512/256 line and the headline.
set -o pipefail
out=gpurun_out/${TAG:-r06p}
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
AVZ_LIB=$D/libavz_dev.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m gpu tests > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
bash tools/gpu_ab_r06.sh ${TAG:-r06p}/ab 2 \
  "base512|AVZ_LIB=$D/libavz.so python bench.py --no-cpu --no-secondary --steps 20 --n-fft 512" \
  "share512|AVZ_LIB=$D/libavz_dev.so python bench.py --no-cpu --no-secondary --steps 20 --n-fft 512" \
  "base|AVZ_LIB=$D/libavz.so python bench.py --no-cpu --no-secondary --steps 20" \
  "share|AVZ_LIB=$D/libavz_dev.so python bench.py --no-cpu --no-secondary --steps 20"
