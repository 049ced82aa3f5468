#!/bin/bash
# rocprofv3 kernel trace + stats of the headline chain at one batch size.
# usage: tools/prof_batch.sh TAG B [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; B=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof_b$B -o run -- \
  python -u bench.py --no-cpu --no-secondary --steps 40 --batch $B "$@" > gpurun_out/$TAG/bench_b$B.log 2>&1
rc=$?
find gpurun_out/$TAG/prof_b$B -name "*kernel_stats.csv" -exec cp {} gpurun_out/$TAG/kernel_stats_b$B.csv \;
find gpurun_out/$TAG/prof_b$B -name "*kernel_trace.csv" -exec cp {} gpurun_out/$TAG/kernel_trace_b$B.csv \;
rm -rf gpurun_out/$TAG/prof_b$B
exit $rc
