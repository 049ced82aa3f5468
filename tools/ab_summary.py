"""Summarise a tools/gpu_ab_r06.sh output directory (one bench JSON per run) as text:
   python tools/ab_summary.py gpurun_out/<tag> [title] > profiles/r06/<name>.txt"""
import glob
import json
import os
import sys

d = sys.argv[1]
title = sys.argv[2] if len(sys.argv) > 2 else d
print(f"# {title}\n# source: {d} (tools/gpu_ab_r06.sh: variants interleaved, one bench.py run each)")
for f in sorted(glob.glob(os.path.join(d, "*.json")), key=lambda p: (p.rsplit("_", 1)[1], p)):
    try:
        line = [x for x in open(f) if x.startswith("{")][-1]
        j = json.loads(line)
    except (IndexError, ValueError):
        continue
    k = j.get("roofline", {}).get("kernels_ms", {})
    name = os.path.basename(f)[:-5]
    print(f"{name:>12s}: {j['value'] / 1e9:7.2f} G  ms/step {j['ms_per_step']:.4f}  " +
          " ".join(f"{n} {v * 1e3:6.1f} us" for n, v in k.items() if v == v and v > 0))
