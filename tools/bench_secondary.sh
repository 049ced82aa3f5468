#!/bin/bash
# Secondary bench lines (parity configs measured with the headline's method): configs[2]
# shard, configs[3] IPD, 512/256, deferred normalisation, configs[4] U-Net.
#   gpurun -- 'bash tools/bench_secondary.sh <tag>'
set -o pipefail
out=gpurun_out/${1:-wl}
mkdir -p $out
i=0
for a in "--batch 512 --interferers 3" "--workload ipd" "--n-fft 512" "--normalize deferred" "--workload unet --steps 3 --warmup 1"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py --no-cpu $a > $out/b$i.log 2>&1 || { tail -5 $out/b$i.log; exit 1; }
  tail -1 $out/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(sys.argv[1], '|', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v*1e3,1) for k,v in r.get('kernels_ms',{}).items()}, {k: round(d[k],1) for k in ('unet_ms','mvdr_chain_ms') if k in d})" "$a"
done
