#!/bin/bash
# Round-5 A/B: HEAD (libavz_A.so) vs the in-kernel piece finalize with the pieces' in-block
# solve (I = libavz.so) over the batch sweep's shapes; the GPU tests on libavz.so first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_len
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/ab_len/tests.log 2>&1 || { tail -40 gpurun_out/ab_len/tests.log; exit 1; }
tail -3 gpurun_out/ab_len/tests.log
REPS=1 bash tools/gpu_ab_r05.sh ab_len256 libavz_A.so libavz_I.so &&
for B in 1 64 257 300; do
  REPS=1 BENCH_ARGS="--batch $B" bash tools/gpu_ab_r05.sh ab_len$B libavz_A.so libavz_I.so || exit 1
done
