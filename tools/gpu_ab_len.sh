#!/bin/bash
# A/B of libavz_A.so (the committed build) against libavz.so (= libavz_I.so, the working
# tree) over the batch sweep's split shapes; the split / fused / timing GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_len
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/ab_len/tests.log 2>&1 || { tail -40 gpurun_out/ab_len/tests.log; exit 1; }
tail -2 gpurun_out/ab_len/tests.log
for B in ${SWEEP:-257 300 1 64}; do
  REPS=1 BENCH_ARGS="--batch $B" bash tools/gpu_ab_r05.sh ab_len$B libavz_A.so libavz_I.so || exit 1
done
