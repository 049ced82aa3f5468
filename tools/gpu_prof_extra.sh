#!/bin/bash
# SQ counters of configs[3]'s IPD kernels and kernel traces of the split batch sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/pmc_sq.sh r05_ipd_sq --no-secondary --workload ipd > /dev/null || exit 1
for B in 257 300; do
  out=gpurun_out/r05_ktrace_b$B
  mkdir -p $out
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
    -- python3 bench.py --no-cpu --no-secondary --steps 20 --batch $B > $out/log 2>&1 || { tail -20 $out/log; exit 1; }
done
