#!/bin/bash
# Full GPU suite on the default library, then an A/B bench of the given alternatives.
#   gpurun -- 'bash tools/gpu_ab_tests.sh <tag> libavz.so lib_alt.so ...'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" $out/gpu_tests.log | head -20; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
bash tools/ab_libs.sh $tag "$@"
