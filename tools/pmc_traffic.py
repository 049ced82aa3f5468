"""Turn rocprofv3 PMC CSVs (separate FETCH_SIZE and WRITE_SIZE passes) into per-launch
HBM traffic of each kernel of the MVDR chain -> profiles/pmc_traffic.json (read by
bench.py for roofline.traffic).

Correction (MI355X_MICROARCH.md section HBM): FETCH_SIZE / WRITE_SIZE are in KiB; on
gfx950 FETCH_SIZE under-counts wide reads (128-B requests tallied at 64 B). Our reads are
4-B-per-lane buffer_load_dword streams, a width the guide leaves uncalibrated; round r01
calibrated x2 on a kernel whose read bytes were known by construction (profiles/r01), and
that factor is applied here. `analysis_read_check` = 2 x FETCH_SIZE of the analysis kernel
over its compulsory input bytes (2 mic + 2 reference streams) shows how tight it is.
Writes are taken as reported.

  python tools/pmc_traffic.py <fetch csv> <write csv> [<fetch csv> <write csv> of the
                               bench with --normalize deferred: the batch-driver path]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the per-utterance synthesis kernel (peak normalisation at N = 1024) folds finalize in:
# then no finalize dispatch exists and its traffic counts 0
KERNELS = {"analysis": ("avz_analysis_kernel",), "solve": ("avz_solve_kernel",),
           "synthesis": ("avz_synthesis_kernel", "avz_synthesis_utt_kernel"),
           "finalize": ("avz_finalize_kernel",)}
B, S, N = 256, 64000, 1024


def per_dispatch(path, counter):
    vals = {k: {} for k in KERNELS}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            for k, pats in KERNELS.items():
                if any(p in name for p in pats):
                    d = int(row["Dispatch_Id"])
                    vals[k][d] = vals[k].get(d, 0.0) + float(row["Counter_Value"])
    return {k: (sum(v.values()) / len(v) if v else 0.0) for k, v in vals.items()}


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    alg_reads = B * 4 * S * 4
    factor = 2.0
    hbm = {k: (factor * fetch[k] + write[k]) * 1024 for k in KERNELS}
    hbm["chain"] = sum(hbm.values())
    n_out = (-(-S // (N // 2))) * (N // 2)
    out = {"kernels": KERNELS, "batch": B, "samples": S, "n_fft": N,
           "fetch_kib_per_launch": fetch, "write_kib_per_launch": write,
           "read_factor": factor, "hbm_bytes_per_launch": hbm,
           "analysis_read_check": factor * fetch["analysis"] * 1024 / alg_reads,
           "alg_bytes_per_launch": {"analysis": alg_reads, "chain": alg_reads + B * n_out * 4},
           "note": "reads = 2 x FETCH_SIZE (gfx950 half-count, calibrated in profiles/r01); "
                   "writes = WRITE_SIZE"}
    if len(sys.argv) >= 5:  # the batch-driver path: normalisation deferred to the consumer
        f2 = per_dispatch(sys.argv[3], "FETCH_SIZE")
        w2 = per_dispatch(sys.argv[4], "WRITE_SIZE")
        h2 = {k: (factor * f2[k] + w2[k]) * 1024 for k in KERNELS}
        h2["chain"] = sum(h2.values())
        out["deferred_hbm_bytes_per_launch"] = h2
        out["deferred_chain_over_alg"] = h2["chain"] / out["alg_bytes_per_launch"]["chain"]
    out["chain_over_alg"] = hbm["chain"] / out["alg_bytes_per_launch"]["chain"]
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
