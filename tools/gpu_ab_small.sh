#!/bin/bash
# A/B of libavz_A.so against libavz_I.so (= libavz.so) at small split batches, both FFT
# sizes; the split-batch parity tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_small
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_fullsize.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/ab_small/tests.log 2>&1 || { tail -40 gpurun_out/ab_small/tests.log; exit 1; }
tail -2 gpurun_out/ab_small/tests.log
for nf in 512 1024; do for B in 1 64; do
  REPS=1 BENCH_ARGS="--batch $B --n-fft $nf" bash tools/gpu_ab_r05.sh ab_small_${nf}_$B libavz_A.so libavz_I.so || exit 1
done; done
