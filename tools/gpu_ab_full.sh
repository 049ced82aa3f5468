#!/bin/bash
# Full default bench line (no CPU baseline) for each library build (AVZ_LIB), same box.
# usage: tools/gpu_ab_full.sh TAG libA.so libB.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
D=real-time-audio-visual-zooming_amd/avz
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  AVZ_LIB=$D/$lib timeout -k 10 400 python -u bench.py --no-cpu ${BENCH_ARGS} \
    > gpurun_out/$TAG/bench_${lib}.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_${lib}.log; exit 1; }
  tail -1 gpurun_out/$TAG/bench_${lib}.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); s=d.get("secondary",{})
print(sys.argv[1], "headline", round(d["value"]/1e9,2), {k: round(v.get("value",0)/1e9,2) for k,v in s.items() if isinstance(v,dict) and "value" in v})' $lib | tee -a gpurun_out/$TAG/summary.txt
done
