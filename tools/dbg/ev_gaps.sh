#!/bin/bash
# Bench with and without the plan's kernel timing (twice each) and a kernel trace of the
# untimed run, to attribute inter-kernel gaps.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-ev2}
mkdir -p $out
for i in 1 2; do
  timeout -k 10 100 python bench.py --no-cpu > $out/t_$i.log 2>&1 || exit 1
  timeout -k 10 100 python bench.py --no-cpu --no-kernel-timing > $out/n_$i.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu --steps 10 --no-kernel-timing > $out/prof.log 2>&1 || exit 1
for f in $out/t_*.log $out/n_*.log; do
  tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1))" $f
done
