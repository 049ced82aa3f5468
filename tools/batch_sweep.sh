#!/bin/bash
# Per-kernel time vs batch size (fixed launch costs vs per-item costs).
set -o pipefail
mkdir -p gpurun_out/sweep
for B in 128 256 512 1024; do
  timeout -k 10 200 python bench.py --no-cpu --steps 10 --batch $B > gpurun_out/sweep/b$B.log 2>&1 || { tail -5 gpurun_out/sweep/b$B.log; exit 1; }
  echo B=$B $(tail -1 gpurun_out/sweep/b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernels_ms"]; print(round(d["value"]/1e9,2), "G", {a: round(v*1e3/d["config"]["batch_per_gpu"],3) for a,v in k.items()}, "us/utt")')
done
