"""GPU: the exact IBM path's certificate constant kappa against decisions and cost.

For configs[1]-generator batches, per kappa: frames and decisions sent to the exact path,
bins whose noise-frame counts differ from the oracle mask (0 = every decision the
reference's, up to count-preserving swaps), and the analysis kernel's time at B = 256.
usage: python tools/dbg/kappa_sweep.py [kappa ...]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "real-time-audio-visual-zooming_amd"))
import avz  # noqa: E402
from avz import synth  # noqa: E402
from oracle import avz_oracle as O  # noqa: E402

kappas = [float(k) for k in sys.argv[1:]] or [0.5, 1, 2, 4, 8, 16, 32, 64, -1]
dev = torch.device("cuda:0")
S = 64000
batches = []
for start, B in ((0, 128), (4242, 256)):
    dm, dt, di = synth.make_batch_device(B, start=start, n_samples=S, n_interferers=2,
                                         device=dev, rng="philox")
    mix, tgt, itf = (x.cpu().numpy() for x in (dm, dt, di))
    msum = np.stack([O.oracle_debug_vec(mix[b], tgt[b], itf[b], n_fft=1024, hop=512, sigma=1.0,
                                        return_stages=True)[1]["mask"].sum(axis=1)
                     for b in range(B)])
    batches.append((start, B, dm, dt, di, msum))
    print(f"oracle for {start}..{start + B - 1} done", flush=True)

for kappa in kappas:
    row = []
    for start, B, dm, dt, di, msum in batches:
        plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                            normalize="peak", max_batch=B, max_samples=S, ibm_kappa=kappa)
        stats = torch.zeros(2, dtype=torch.int64, device=dev)
        plan.set_ibm_stats(stats)
        cov = torch.zeros((B, 513, 5), dtype=torch.float64, device=dev)
        plan.run(dm, ref_tgt=dt, ref_int=di, cov_out=cov)
        torch.cuda.synchronize()
        plan.set_ibm_stats(None)
        bad = int(np.sum(cov[:, :, 4].cpu().numpy() != msum))
        ms = float("nan")
        if B == 256:
            for _ in range(5):
                plan.run(dm, ref_tgt=dt, ref_int=di)
            plan.set_timing(True)
            for _ in range(20):
                plan.run(dm, ref_tgt=dt, ref_int=di)
            t = plan.timing()
            plan.set_timing(False)
            ms = t["analysis"]
        row.append(f"[{start}+{B}] frames {int(stats[0])} ({int(stats[0]) / (B * 126):.3%}) "
                   f"decisions {int(stats[1])} bad bins {bad}"
                   + (f" analysis {ms * 1e3:.1f} us" if B == 256 else ""))
    print(f"kappa {kappa:g}: " + "; ".join(row), flush=True)
