#!/bin/bash
# GPU test run on the box: selected test files (default: all GPU tests), verbose log.
#   gpurun -- 'bash tools/gpu_tests.sh <tag> [pytest args...]'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
args=${@:-tests}
timeout -k 10 600 python -u -m pytest $args -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|max \||istft|hybrid:" $out/gpu_tests.log | tail -60
exit $rc
