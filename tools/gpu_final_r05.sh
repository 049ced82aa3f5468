#!/bin/bash
# Round-5 final build on the GPU: every GPU test, the round profile (kernel stats, PMC
# traffic, the bench line) and the SQ counters of the headline kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r05f}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$tag/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$tag/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$tag/gpu_tests.log
bash tools/profile_round.sh $tag && bash tools/pmc_sq.sh ${tag}_sq --no-secondary
