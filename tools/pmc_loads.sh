#!/bin/bash
# Load-path attribution of the chain kernels: SQ issue/wait counters
# of vector-memory instructions, texture address (TA) / data (TD) unit busy cycles and the
# vector L1 (TCP) request/stall counters, each group in its own --pmc pass (slot limits:
# 8 SQ, 2 TA, 2 TD, 4 TCP), headline configuration only.
#   gpurun -- 'bash tools/pmc_loads.sh <tag>'
set -o pipefail
tag=${1:-loads}
shift || true
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
have() { grep -qw "$1" $out/counters_list.txt; }
pick() { local r=""; for c in "$@"; do have $c && r="$r $c"; done; echo $r; }
P1=$(pick SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY)
P2=$(pick TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY TD_LOAD_WAVEFRONT)
P3=$(pick TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES)
P4=$(pick GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS)
echo "passes: [$P1] [$P2] [$P3] [$P4]" | tee $out/passes.txt
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  [ -z "$P" ] && continue
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $out/p$i -o run \
    -- python3 bench.py --no-cpu --no-secondary --steps 5 --warmup 2 --no-kernel-timing "$@" > $out/p$i.log 2>&1 || { tail -20 $out/p$i.log; exit 1; }
done
python3 - $out <<'PY' | tee $out/load_counters.txt
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(out + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "avz" not in n or "scene" in n or "metrics" in n:
            continue
        k = n.split("(")[0].replace("void avz::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, c in agg.items():
    print(k)
    for x in sorted(c):
        print(f"   {x:28s} {c[x] / len(disp[(k, x)]):16.0f}")
PY
