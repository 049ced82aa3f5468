set -o pipefail
out=gpurun_out/${1:-bc}; mkdir -p $out
t0=$(date +%s); timeout -k 10 400 python bench.py > $out/bench.log 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
python3 - $out/bench.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]/1e9, 2), "G ms", round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 3))
print("kernels", {k: round(v*1e3, 1) for k, v in d["roofline"]["kernels_ms"].items()})
print("cpu", d["cpu_baseline"]["cores"], d["cpu_baseline"]["cores_available"], round(d["cpu_baseline"]["value"]/1e6, 1), "M")
for k, v in d.get("secondary", {}).items():
    if "error" in v: print(k, v); continue
    print(k, round(v["value"]/1e9, 2), "G", round(v["ms_per_step"], 4), "ms frac", round(v["frac"], 3), {a: round(b*1e3, 1) for a, b in v.get("kernels_ms", {}).items()})
print("sir", d["sir"])
PY
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rehearse-shared-gpu --steps 5 > $out/n2.log 2> $out/n2.err || { tail -20 $out/n2.err; exit 1; }
tail -1 $out/n2.log | cut -c1-400
