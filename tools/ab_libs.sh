#!/bin/bash
# A/B of alternative builds of libavz.so on the GPU box: bench line + per-kernel times
# for each library, optionally the GPU test suite against the first alternative.
#   gpurun -- 'bash tools/ab_libs.sh <tag> [--tests] lib1.so lib2.so ...'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
tests=0
if [ "$1" = "--tests" ]; then tests=1; shift; fi
D=real-time-audio-visual-zooming_amd/avz
if [ $tests = 1 ]; then
  AVZ_LIB=$D/$1 timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests_$1.log 2>&1 || { tail -30 $out/gpu_tests_$1.log; exit 1; }
  tail -1 $out/gpu_tests_$1.log
fi
for rep in $(seq 1 ${REPS:-2}); do
for lib in "$@"; do
  AVZ_LIB=$D/$lib timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS} > $out/bench_${lib}_$rep.log 2>&1 || { tail -20 $out/bench_${lib}_$rep.log; exit 1; }
  tail -1 $out/bench_${lib}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], round(d["value"]/1e9,2), "G ms/step", round(d["ms_per_step"],4), {k: round(v*1e3,1) for k,v in r.get("kernels_ms",{}).items()}, "dominant", round(r.get("dominant_kernel",{}).get("kernel_ms",0)*1e3,1))' $lib
done
done
