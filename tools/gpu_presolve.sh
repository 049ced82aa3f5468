#!/bin/bash
# Pre-solve with bin N/2 spread over a wave: GPU tests, A/B at split batch sizes (1024/512),
# configs[0] latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/presolve
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/presolve/tests.log 2>&1 || { tail -40 gpurun_out/presolve/tests.log; exit 1; }
tail -2 gpurun_out/presolve/tests.log
for B in 1 16 257 300; do
  REPS=1 BENCH_ARGS="--batch $B" bash tools/gpu_ab_r05.sh presolve_$B libavz_A.so libavz_I.so || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu --secondary "configs[0]_latency" > gpurun_out/presolve/lat.log 2>&1
