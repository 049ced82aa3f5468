#!/bin/bash
# GPU tests on the default library, then full default bench lines (every secondary) per library.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in $(seq 1 ${REPS:-2}); do
for lib in "$@"; do
  AVZ_LIB=$D/$lib timeout -k 10 300 python bench.py --no-cpu > $out/bench_${lib}_$rep.log 2>&1 || { tail -20 $out/bench_${lib}_$rep.log; exit 1; }
  tail -1 $out/bench_${lib}_$rep.log | python3 -c '
import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]
print(sys.argv[1], round(d["value"]/1e9,2), "G", {k: round(v*1e3,1) for k,v in r["kernels_ms"].items()}, "dom", round(r["dominant_kernel"]["kernel_ms"]*1e3,1))
print("   ", {k: (round(v["value"]/1e9,1), round(v.get("kernels_ms",{}).get("analysis",0)*1e3,1)) for k,v in d.get("secondary",{}).items()})' $lib
done
done
