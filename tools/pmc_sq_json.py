"""SQ / GRBM counter passes of tools/pmc_sq.sh -> profiles/pmc_sq.json: per kernel of the
bench chain the per-dispatch averages, read by bench.py for the roofline entries' VALU and
LDS busy fractions:
  valu_busy = SQ_ACTIVE_INST_VALU x 4 / (4 SIMDs x CUs) / (GRBM_GUI_ACTIVE / 8 XCDs)
  lds_busy  = SQ_LDS_IDX_ACTIVE / CUs / (GRBM_GUI_ACTIVE / 8 XCDs)
(SQ_ACTIVE_INST_* count in 4-cycle units -- the gfx94x VALUBusy formula; GRBM_GUI_ACTIVE is
the sum over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'; SQ_LDS_IDX_ACTIVE: LDS-array
cycles per CU.)
  python tools/pmc_sq_json.py <pmc_sq.sh output dir> [bench args: --batch B ...]
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = sys.argv[1]
    args = sys.argv[2:]
    batch = int(args[args.index("--batch") + 1]) if "--batch" in args else 256
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
    kernels = {k: {x: c[x] / len(disp[(k, x)]) for x in c} for k, c in agg.items()}
    doc = {"batch": batch, "n_fft": 1024, "samples": 64000, "source": os.path.relpath(out, ROOT),
           "formula": {"valu_busy": "SQ_ACTIVE_INST_VALU*4/(4*CUs)/(GRBM_GUI_ACTIVE/8)",
                       "lds_busy": "SQ_LDS_IDX_ACTIVE/CUs/(GRBM_GUI_ACTIVE/8)"},
           "kernels": kernels}
    path = os.path.join(ROOT, "profiles", "pmc_sq.json")
    json.dump(doc, open(path, "w"), indent=1)
    print(f"wrote {path}: {len(kernels)} kernels")


if __name__ == "__main__":
    main()
