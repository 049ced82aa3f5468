#!/bin/bash
# Headline sensitivity to GPU warm-up after the CPU baseline (default bench = CPU baseline,
# then 5 warmup steps); alternating --warmup 5 and --warmup 200.
set -o pipefail
out=gpurun_out/warm
mkdir -p $out
for i in 1 2; do
  for w in 5 200; do
    timeout -k 10 200 python bench.py --warmup $w > $out/w${w}_$i.log 2>&1 || exit 1
    tail -1 $out/w${w}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup', sys.argv[1], round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1))" $w
  done
done
