#!/bin/bash
# GPU test run + default bench on the box, each step under its own time limit; stops at
# the first failure.   gpurun -- 'bash tools/gpu_check.sh <tag> [bench args...]'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $out/gpu_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err
rc=$?
tail -c 600 $out/bench.json
exit $rc
