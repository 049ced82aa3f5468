#!/bin/bash
# smoke() + repeated default bench lines at HEAD (headline variance)
set -o pipefail
out=gpurun_out/${1:-var}
mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu --no-secondary > $out/bench_$i.log 2>&1 || { tail -20 $out/bench_$i.log; exit 1; }
  tail -1 $out/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e9,2), "G ms/step", round(d["ms_per_step"],4), {k: round(v*1e3,1) for k,v in r["kernels_ms"].items()}, "dominant", round(r["dominant_kernel"]["kernel_ms"]*1e3,1), "frac", round(r["frac"],3))'
done
