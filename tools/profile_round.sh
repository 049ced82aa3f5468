#!/bin/bash
# Round profile on the GPU box (headline kernels with --no-secondary): kernel trace/stats of the bench, two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE; never combined with runtime/sys traces), traffic json,
# the bench line itself. Output under gpurun_out/<tag>/ ; copy what is judged to profiles/.
#   gpurun -- 'bash tools/profile_round.sh r03a'
set -o pipefail
tag=${1:-prof}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ktrace -o run \
  -- python3 bench.py --no-cpu --no-secondary --steps 20 > $out/ktrace.log 2>&1 || { tail -20 $out/ktrace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run \
  -- python3 bench.py --no-cpu --steps 5 --warmup 2 --no-kernel-timing --no-secondary > $out/pmc_fetch.log 2>&1 || { tail -20 $out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run \
  -- python3 bench.py --no-cpu --steps 5 --warmup 2 --no-kernel-timing --no-secondary > $out/pmc_write.log 2>&1 || { tail -20 $out/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch_d -o run \
  -- python3 bench.py --no-cpu --steps 5 --warmup 2 --no-kernel-timing --no-secondary --normalize deferred > $out/pmc_fetch_d.log 2>&1 || { tail -20 $out/pmc_fetch_d.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write_d -o run \
  -- python3 bench.py --no-cpu --steps 5 --warmup 2 --no-kernel-timing --no-secondary --normalize deferred > $out/pmc_write_d.log 2>&1 || { tail -20 $out/pmc_write_d.log; exit 1; }
f1=$(find $out/pmc_fetch -name "*counter_collection.csv" | head -1)
f2=$(find $out/pmc_write -name "*counter_collection.csv" | head -1)
f3=$(find $out/pmc_fetch_d -name "*counter_collection.csv" | head -1)
f4=$(find $out/pmc_write_d -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$f1" "$f2" "$f3" "$f4" > $out/pmc_traffic.log 2>&1 || { cat $out/pmc_traffic.log; exit 1; }
cp profiles/pmc_traffic.json $out/
timeout -k 10 300 python bench.py --no-cpu > $out/bench_traffic.log 2>&1 || { tail -20 $out/bench_traffic.log; exit 1; }
tail -1 $out/bench_traffic.log
# every configuration of the default line (secondaries included: avz_spectral_kernel's row)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ktrace_all -o run \
  -- python3 bench.py --no-cpu --steps 10 > $out/ktrace_all.log 2>&1 || { tail -20 $out/ktrace_all.log; exit 1; }
f=$(find $out/ktrace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "avz" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
