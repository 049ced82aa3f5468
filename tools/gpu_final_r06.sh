#!/bin/bash
# Round-6 final build on the GPU: the round profile (kernel stats, PMC traffic, the bench
# line) and the SQ counters of the headline kernels (profiles/pmc_sq.json for bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r06f}
mkdir -p gpurun_out/$tag
bash tools/pmc_sq.sh ${tag}_sq --no-secondary && cp profiles/pmc_sq.json gpurun_out/${tag}_sq/ && \
bash tools/profile_round.sh $tag
