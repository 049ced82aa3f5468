"""In-process A/B of the synthesis paths (plan.set_diagnostics synth_variant: 1 per-utterance
kernel, 0 chunk grid + finalize) on configs[1]
(and optionally other workloads): outputs of the variants compared element-wise, then
per-kernel HIP-event times over alternating rounds.

    python tools/ab_synth.py [--batch 256] [--rounds 3] [--calls 30] [--workload ibm|ipd]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "real-time-audio-visual-zooming_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import avz  # noqa: E402
from avz import synth  # noqa: E402
from avz._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--workload", default="ibm")
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--normalize", default="peak")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, S = a.batch, 64000
    mix, tgt, itf = synth.make_batch_device(B, start=0, n_samples=S, n_interferers=2, device=dev,
                                            rng="philox")
    if a.workload == "ibm":
        plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                            normalize=a.normalize, max_batch=B, max_samples=S)
        refs = dict(ref_tgt=tgt, ref_int=itf)
    else:
        plan = avz.MVDRPlan(n_fft=1024, sigma=1e-7, mic_d=0.01, mask="ipd", postfilter="none",
                            normalize=a.normalize, norm_eps=1e-6, max_batch=B, max_samples=S)
        refs = {}
    lens = torch.full((B,), S, dtype=torch.int32, device=dev)
    out = plan.alloc_out(B, S, dev)
    peak = torch.empty((B,), dtype=torch.float32, device=dev)
    variants = [int(v) for v in a.variants.split(",")]
    res = {}
    for v in variants:
        plan.set_diagnostics(synth_variant=v)
        plan.run(mix, lens, max_len=S, out=out, peak=peak, **refs)
        torch.cuda.synchronize()
        res[v] = (out.clone(), peak.clone())
    n = plan.out_len(S)
    o0, p0 = res[variants[0]]
    for v in variants[1:]:
        o, p = res[v]
        d = (o[:, :n] - o0[:, :n]).abs().max().item()
        dp = ((p - p0).abs() / p0.abs().clamp_min(1e-30)).max().item()
        print(f"variant {v} vs {variants[0]}: max|out diff| = {d:.3e}, max rel peak diff = {dp:.3e}, "
              f"finite {bool(torch.isfinite(o[:, :n]).all())}")
    # warm the clock
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        plan.run(mix, lens, max_len=S, out=out, peak=peak, **refs)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for v in variants:
            plan.set_diagnostics(synth_variant=v)
            for _ in range(5):
                plan.run(mix, lens, max_len=S, out=out, peak=peak, **refs)
            plan.set_timing(True)
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            for _ in range(a.calls):
                plan.run(mix, lens, max_len=S, out=out, peak=peak, **refs)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - w0) / a.calls
            t = plan.timing()
            plan.set_timing(False)
            print(f"round {r} variant {v}: " + " ".join(f"{k} {t[k] * 1e3:.1f}" for k in plan.KERNELS)
                  + f" us; wall {wall * 1e6:.1f} us/call (events on)", flush=True)
    plan.set_diagnostics(synth_variant=2)  # the shipped default


if __name__ == "__main__":
    main()
