#!/bin/bash
# Default bench line (every secondary configuration) without the CPU baseline, summarised.
#   gpurun -- 'bash tools/bench_full.sh <tag>'
set -o pipefail
out=gpurun_out/${1:-full}
mkdir -p $out
timeout -k 10 400 python bench.py --no-cpu > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | python3 -c '
import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]
print(round(d["value"]/1e9,2), "G", {k: round(v*1e3,1) for k,v in r["kernels_ms"].items()}, "dom", round(r["dominant_kernel"]["kernel_ms"]*1e3,1))
for k,v in d.get("secondary",{}).items():
    print(k, round(v["value"]/1e9,2), {a: round(b*1e3,1) for a,b in v.get("kernels_ms",{}).items()})'
