"""Turn rocprofv3 PMC CSVs (separate FETCH_SIZE and WRITE_SIZE passes) into per-launch
HBM traffic of the fused kernel -> profiles/pmc_traffic.json (read by bench.py).

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (128-B requests tallied at
64 B). Our loads are 4 B/lane buffer_load_dword (a width the guide lists as
uncalibrated); calibration against the design's known byte count: with x2 the read
side equals algorithmic reads + the pass-2 mix re-read + the normalisation re-read
(262 + 131 + 65 = 458 MB at B = 256) to <1 %, so `hbm_bytes_per_launch` uses
2 x FETCH_SIZE + WRITE_SIZE.

  python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, counter):
    vals = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if "avz_fused_kernel" not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = int(row["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    B, S, N = 256, 64000, 1024
    alg = B * (4 * S * 4 + S * 4)
    out = {"kernel": "avz_fused_kernel<1024,IBM,512>", "batch": B, "samples": S, "n_fft": N,
           "dispatches": [len(fetch), len(write)],
           "fetch_kib_per_launch": f_kib, "write_kib_per_launch": w_kib,
           "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024,
           "hbm_bytes_per_launch_raw": (f_kib + w_kib) * 1024,
           "alg_bytes_per_launch": alg,
           "read_correction": "2 x FETCH_SIZE (gfx950 half-count; calibrated vs known bytes)"}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
