#!/bin/bash
# A/B of library builds (AVZ_LIB) on one box: the headline bench line's kernels, REPS rounds.
# usage: tools/gpu_ab_r05.sh TAG libA.so libB.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
D=real-time-audio-visual-zooming_amd/avz
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    AVZ_LIB=$D/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-secondary --steps 40 ${BENCH_ARGS} \
      > gpurun_out/$TAG/bench_${lib}_$rep.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_${lib}_$rep.log; exit 1; }
    tail -1 gpurun_out/$TAG/bench_${lib}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], round(d["value"]/1e9,2), "G ms/step", round(d["ms_per_step"],4), {k: round(v*1e3,1) for k,v in r.get("kernels_ms",{}).items()})' $lib | tee -a gpurun_out/$TAG/summary.txt
  done
done
