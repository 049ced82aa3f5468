"""GPU: test_external_mask_equals_ibm_mode's configuration, diagnosed -- IBM-mode noise counts
(cov_out column 4) of the chunked driver's items against the oracle target mask's, and the
IBM vs external-mask waveform difference, per kappa.
usage: python tools/dbg/hybrid_ibm_check.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-audio-visual-zooming_amd"), os.path.join(ROOT, "tests")]
from conftest import triple_f32  # noqa: E402
from oracle import avz_oracle as O  # noqa: E402
from avz import final_pipeline as fp  # noqa: E402
import avz  # noqa: E402

d = torch.device("cuda:0")
mix, t, i = triple_f32("test", seg=(0, 48000))
S = mix.shape[1]
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(d)  # noqa: E731
masks = np.stack([O.chunk_target_mask(t, i, s) for s in range(0, S, 16000)])
for kappa in (-1.0, 16.0, 1e30):
    ibm = fp.ChunkedHybridBeamformer(max_items=3, mask="ibm")
    pl = ibm.plan
    kw = {k: getattr(pl.cfg, k) for k in pl.cfg.__dataclass_fields__} if hasattr(pl.cfg, "__dataclass_fields__") else None
    if kw is not None:
        kw["ibm_kappa"] = kappa
        ibm.plan = avz.MVDRPlan(**kw)
    y0, _ = ibm.run(T(mix)[None], ref_tgt=T(t)[None], ref_int=T(i)[None])
    ext = fp.ChunkedHybridBeamformer(max_items=3, mask="external")
    y1, _ = ext.run(T(mix)[None], mask_fn=lambda items: T(masks))
    torch.cuda.synchronize()
    print(f"kappa {kappa:g}: max|y_ibm - y_ext| {float((y0 - y1).abs().max()):.3e}", flush=True)
