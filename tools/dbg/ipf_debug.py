"""Diagnose the in-kernel piece finalize: B = 257 runs in modes 0, 1, 2, 0; per utterance,
the sample ranges (valid part only) where runs differ, and the ratio there."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-audio-visual-zooming_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import avz  # noqa: E402
from avz import synth  # noqa: E402
from avz._lib import lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 257
S = 64000
dev = torch.device("cuda:0")
dm, dt, di = synth.make_batch_device(B, start=77, n_samples=S, n_interferers=2, device=dev,
                                     rng="philox")
lens = np.full(B, S, np.int32)
lens[2::5] = np.random.default_rng(B).integers(1024, S + 1, size=len(lens[2::5]))
lt = torch.from_numpy(lens).to(dev)
plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                    normalize="peak", max_batch=B, max_samples=S)
runs = []
for mode in (0, 0, 1, 2, 0):
    plan.set_diagnostics(ipf_mode=mode)
    out, peak = plan.run(dm, lt, max_len=S, ref_tgt=dt, ref_int=di)
    torch.cuda.synchronize()
    runs.append((mode, out.clone().cpu().numpy(), peak.clone().cpu().numpy()))
plan.set_diagnostics(ipf_mode=0)
n_out = plan.out_len(S)
ref = runs[1][1]
for (mode, o, p) in runs:
    bad = []
    for b in range(B):
        n = plan.out_len(int(lens[b]))
        a, r = o[b, :n], ref[b, :n]
        d = np.nonzero(~((a == r) | (np.isnan(a) & np.isnan(r))))[0]
        if len(d):
            seg = sorted(set((d // 512).tolist()))
            ratio = np.median(a[d] / np.where(r[d] == 0, np.nan, r[d]))
            bad.append((b, int(lens[b]), len(d), seg[:12], float(ratio), float(np.abs(a[:n]).max()),
                        float(np.abs(r[:n]).max())))
    print(f"mode {mode}: {len(bad)} utterances differ from run 1")
    for x in bad[:12]:
        print("   ", x)
