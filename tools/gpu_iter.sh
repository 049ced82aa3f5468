#!/bin/bash
# One GPU iteration: parity tests, bench line, per-kernel rocprofv3 stats, phase stamps.
# Run on the GPU box:  gpurun -- 'bash tools/gpu_iter.sh [tag]'
set -o pipefail
tag=${1:-iter}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 240 python bench.py --no-cpu > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["value"]/1e9,2), "G", d["unit"], "ms/step", round(d["ms_per_step"],4))'
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu --steps 10 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "avz" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
if [ -f real-time-audio-visual-zooming_amd/avz/libavz_stamps.so ]; then
  timeout -k 10 200 python tools/phase_profile.py > $out/phase.log 2>&1 && grep -v amdgpu.ids $out/phase.log
fi
