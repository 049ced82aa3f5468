#!/bin/bash
# Round check on the GPU box: full GPU suite, then the round profile (bench, kernel
# stats, PMC traffic of the headline and the deferred-normalisation path).
#   gpurun -- 'bash tools/gpu_round.sh <tag>'
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $out/gpu_tests.log | head; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
bash tools/profile_round.sh $tag
