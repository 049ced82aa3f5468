#!/bin/bash
# Synthesis-path A/B (tools/ab_synth.py) then, optionally, the GPU test suite on the
# default build.   gpurun -- 'bash tools/gpu_ab_synth.sh <tag> [--tests] [ab args...]'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
tests=0
if [ "$1" = "--tests" ]; then tests=1; shift; fi
timeout -k 10 150 python -u tools/ab_synth.py "$@" > $out/ab_synth.log 2>&1
rc=$?
grep -v amdgpu.ids $out/ab_synth.log
[ $rc -ne 0 ] && exit $rc
if [ $tests = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > $out/gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" $out/gpu_tests.log | tail -20
fi
exit $rc
