#!/bin/bash
# Small batches after the lanes-per-bin solve: every GPU test, the small-batch A/B and the
# configs[0] latency entry.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/small2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/small2/tests.log 2>&1 || { tail -40 gpurun_out/small2/tests.log; exit 1; }
tail -2 gpurun_out/small2/tests.log
for nf in 512 1024; do for B in 1 16; do
  REPS=1 BENCH_ARGS="--batch $B --n-fft $nf" bash tools/gpu_ab_r05.sh small2_${nf}_$B libavz_A.so libavz_I.so || exit 1
done; done
timeout -k 10 300 python -u bench.py --no-cpu --secondary "configs[0]_latency" > gpurun_out/small2/lat.log 2>&1
