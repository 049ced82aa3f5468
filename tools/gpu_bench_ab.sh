#!/bin/bash
# Default bench line under each synthesis variant (AVZ_SYNTH_VARIANT), REPS rounds.
#   gpurun -- 'bash tools/gpu_bench_ab.sh <tag> [variants...]'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for rep in $(seq 1 ${REPS:-1}); do
for v in "$@"; do
  AVZ_SYNTH_VARIANT=$v timeout -k 10 400 python bench.py --no-cpu ${BENCH_ARGS} > $out/bench_v${v}_$rep.json 2> $out/bench_v${v}_$rep.err || { tail -5 $out/bench_v${v}_$rep.err; exit 1; }
  python3 - $out/bench_v${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("variant", sys.argv[2], round(d["value"] / 1e9, 2), "G", round(d["ms_per_step"] * 1e3, 1), "us/step",
      {k: round(v * 1e3, 1) for k, v in r.get("kernels_ms", {}).items()})
for k, e in d.get("secondary", {}).items():
    if "value" in e:
        print("   ", k, round(e["value"] / 1e9, 2), "G", round(e["ms_per_step"] * 1e3, 1), "us/step",
              {kk: round(vv * 1e3, 1) for kk, vv in e.get("kernels_ms", {}).items()})
PY
done
done
