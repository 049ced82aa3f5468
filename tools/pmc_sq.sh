#!/bin/bash
# SQ counters (issue/stall breakdown) of the bench kernels, separate --pmc passes.
#   gpurun -- 'bash tools/pmc_sq.sh <tag> [extra bench.py args]'
set -o pipefail
tag=${1:-sq}
shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $out/p$i -o run \
    -- python3 bench.py --no-cpu --steps 5 --warmup 2 --no-kernel-timing "$@" > $out/p$i.log 2>&1 || { tail -20 $out/p$i.log; exit 1; }
done
python3 - $out <<'PY' | tee $out/sq_counters.txt
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
        print(f"   {x:24s} {c[x] / len(disp[(k, x)]):16.0f}")
PY
# per-dispatch averages -> profiles/pmc_sq.json (bench.py's valu_busy / lds_busy)
python3 tools/pmc_sq_json.py $out "$@" || exit 1
