#!/bin/bash
# GPU tests on the default library, N = 512 A/B against the pre-interleave build, and the
# wave-0 (mic) / wave-2 (reference) phase stamps of the IBM analysis + synthesis.
set -o pipefail
out=gpurun_out/${1:-r03d}
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for w in 0 2; do
  AVZ_LIB=$D/libavz_st$w.so timeout -k 10 200 python tools/phase_profile.py > $out/stamps_wave$w.txt 2>&1 || { tail -20 $out/stamps_wave$w.txt; exit 1; }
  echo "== wave $w"; grep -v amdgpu.ids $out/stamps_wave$w.txt
done
REPS=2 BENCH_ARGS="--no-secondary --n-fft 512" bash tools/ab_libs.sh ${1:-r03d}_512 libavz.so libavz_il0.so
