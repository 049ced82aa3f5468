#!/bin/bash
# All bench workloads on the GPU box (configs[1] default line, configs[3] ipd, configs[4] unet).
#   gpurun -- 'bash tools/bench_workloads.sh <tag>'
set -o pipefail
tag=${1:-wl}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python bench.py > $out/bench_ibm.log 2>&1 || { tail -20 $out/bench_ibm.log; exit 1; }
tail -1 $out/bench_ibm.log
timeout -k 10 300 python bench.py --workload ipd > $out/bench_ipd.log 2>&1 || { tail -20 $out/bench_ipd.log; exit 1; }
tail -1 $out/bench_ipd.log
timeout -k 10 400 python bench.py --workload unet --steps 3 --warmup 1 > $out/bench_unet.log 2>&1 || { tail -20 $out/bench_unet.log; exit 1; }
tail -1 $out/bench_unet.log
