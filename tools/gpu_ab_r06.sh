#!/bin/bash
# Same-box A/B of bench lines: gpurun -- 'bash tools/gpu_ab_r06.sh <tag> <reps> "<name>|<cmd>" ...'
# each cmd is run reps times, interleaved; prints value and kernel ms per run.
set -o pipefail
tag=$1; reps=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    name=${spec%%|*}; cmd=${spec#*|}
    timeout -k 10 300 bash -c "$cmd" > $out/${name}_$rep.json 2> $out/${name}_$rep.err || { tail -5 $out/${name}_$rep.err; exit 1; }
    python3 - $out/${name}_$rep.json $name <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:>10s}: {d['value'] / 1e9:7.2f} G  ms/step {d['ms_per_step']:.4f}  " +
      " ".join(f"{n} {v * 1e3:6.1f}" for n, v in k.items()), flush=True)
PY
  done
done
