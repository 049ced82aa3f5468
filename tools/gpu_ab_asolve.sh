#!/bin/bash
# Staged partials (or any candidate): every GPU test on libavz.so (= libavz_I.so), then A/B against
# libavz_A.so on the configurations with >= 2 synthesis rounds and the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/asolve
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/asolve/tests.log 2>&1 || { tail -40 gpurun_out/asolve/tests.log; exit 1; }
tail -2 gpurun_out/asolve/tests.log
REPS=2 BENCH_ARGS="--workload ipd" bash tools/gpu_ab_r05.sh ab_as_ipd libavz_A.so libavz_I.so &&
REPS=2 BENCH_ARGS="--batch 512 --interferers 3" bash tools/gpu_ab_r05.sh ab_as_512 libavz_A.so libavz_I.so &&
REPS=2 bash tools/gpu_ab_r05.sh ab_as_256 libavz_A.so libavz_I.so
