"""Exact-path work-sharing trace (diagnostic build libavz_xt.so, -DAVZ_XTRACE): per analysis
block the loop end, own-unit end and exit times (s_memrealtime, 100 MHz) relative to the
earliest block start, the pieces it ran, the units it published; one launch of configs[1].

  AVZ_LIB=.../libavz_xt.so python tools/xtrace.py [--start 0] [--kappa 16]
"""
import argparse
import ctypes as ct
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-audio-visual-zooming_amd")]
os.environ.setdefault("AVZ_LIB", os.path.join(ROOT, "real-time-audio-visual-zooming_amd", "avz",
                                              "libavz_xt.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import avz  # noqa: E402
from avz import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--start", type=int, default=0)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--kappa", type=float, default=None)
a = ap.parse_args()
S = 64000
dev = torch.device("cuda:0")
mix, tgt, itf = synth.make_batch_device(a.batch, start=a.start, n_samples=S, n_interferers=2,
                                        device=dev, rng="philox")
plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                    normalize="peak", max_batch=a.batch, max_samples=S,
                    **({"ibm_kappa": a.kappa} if a.kappa is not None else {}))
st = torch.zeros((4096, 16), dtype=torch.int64, device=dev)
lib = avz._lib.lib
setter = lib.avz_debug_set_stamps_chunked
setter.argtypes = [ct.c_void_p]
for _ in range(3):
    plan.run(mix, ref_tgt=tgt, ref_int=itf)
torch.cuda.synchronize()
for rep in range(2):
    st.zero_()
    assert setter(ct.c_void_p(st.data_ptr())) == 0
    plan.run(mix, ref_tgt=tgt, ref_int=itf)
    torch.cuda.synchronize()
    assert setter(ct.c_void_p(0)) == 0
    x = st.cpu().numpy()
    x = x[x[:, 0] > 0]
    t0 = x[:, 0].min()
    us = lambda v: (v.astype(np.float64) - t0) / 100.0  # noqa: E731
    loop, own, end = us(x[:, 1]), us(x[:, 2]), us(x[:, 3])
    print(f"== launch {rep}: {len(x)} blocks; loop end {loop.min():.1f}-{loop.max():.1f} "
          f"(median {np.median(loop):.1f}) us; exit max {end.max():.1f} us")
    npc = x[:, 4]
    print(f"pieces per block: {np.bincount(npc).tolist()}; published units "
          f"{int((x[:, 13] % 256).sum())}, their pieces {int((x[:, 13] // 256).sum())}")
    pc = x[:, 4] > 0
    ph = x[pc][:, 8:12].sum(axis=0) / 100.0 / max(1, int(x[pc][:, 4].sum()))
    print("round phases per piece (us): loads+ref A %.1f, ref B + barrier %.1f, mic FFT + barrier "
          "%.1f, bins + barrier %.1f; claim total per block mean %.1f max %.1f; tables mean %.1f"
          % (*ph, x[:, 14].mean() / 100, x[:, 14].max() / 100, x[pc][:, 15].mean() / 100))
    npcs = max(1, int(x[pc][:, 4].sum()))
    pub = x[:, 13] % 256 > 0
    print("per piece: finish (barrier, release, arrival) %.1f us, merge %.1f us; publish per unit %.1f us"
          % (x[pc][:, 6].sum() / 100 / npcs, x[pc][:, 7].sum() / 100 / npcs,
             x[pub][:, 12].sum() / 100 / max(1, int((x[pub][:, 13] % 256).sum()))))
    pubm = x[:, 13] % 256 > 0
    for name, m in (("publishers", pubm), ("others", ~pubm)):
        if m.any():
            print(f"loop end of {name} ({int(m.sum())}): p10 {np.percentile(loop[m], 10):.1f} "
                  f"p50 {np.percentile(loop[m], 50):.1f} p90 {np.percentile(loop[m], 90):.1f} "
                  f"max {loop[m].max():.1f} us")
    order = np.argsort(-end)[:8]
    for i in order:
        print(f"  blk {i:4d}: start {us(x[i:i+1, 0])[0]:6.1f} loop {loop[i]:6.1f} own {own[i]:6.1f} "
              f"exit {end[i]:6.1f}  pieces {x[i, 4]} ({x[i, 5] / 100:.1f} us) "
              f"finish {x[i, 6] / 100:.1f} merge {x[i, 7] / 100:.1f} "
              f"claim {x[i, 14] / 100:.1f} tables {x[i, 15] / 100:.1f} "
              f"published {x[i, 13] % 256} ({x[i, 12] / 100:.1f} us)")
