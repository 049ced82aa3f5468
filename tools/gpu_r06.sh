#!/bin/bash
# Round-6 GPU session steps: gpurun -- 'bash tools/gpu_r06.sh <tag> <step>...'
#   tests:<pytest args>  bench[:args]  prof[:args]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export PYTHONUNBUFFERED=1
for step in "$@"; do
  case $step in
    tests:*)
      t=${step#tests:}
      timeout -k 10 900 python -u -m pytest $t -x -v -s --timeout 300 --timeout-method thread \
        > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
      tail -5 $out/tests.log ;;
    bench*)
      a=${step#bench}; a=${a#:}
      timeout -k 10 600 python bench.py $a > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
      tail -c 3000 $out/bench.json ;;
    prof*)
      a=${step#prof}; a=${a#:}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py $a > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
      find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \; ;;
  esac
done
