"""Per-phase time breakdown of the MVDR kernels (diagnostic build libavz_stamps.so).

Wave 0 of every block accumulates s_memrealtime (100 MHz) deltas between the
kernel's barriers; this prints the mean per block in microseconds. The stamped build
has extra scalar work in wave 0, so read the SHARES, not the absolute total.

  AVZ_LIB=.../libavz_stamps.so python tools/phase_profile.py [--batch 256] [--mask ibm]
"""
import argparse
import ctypes as ct
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-audio-visual-zooming_amd")]
os.environ.setdefault("AVZ_LIB", os.path.join(ROOT, "real-time-audio-visual-zooming_amd", "avz",
                                              "libavz_stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import avz  # noqa: E402
from avz import synth  # noqa: E402

# avz_chunked.hip stamp slots: analysis 0-3, 11, 12; synthesis 4-10; the role-split
# synthesis (--rs): producer wave 4-7, consumer wave 8-10, 13-15
PHASES = ["A load wait", "A barrier 1", "A barrier 2", "A window+FFT", "S prologue",
          "S load wait", "S FFT", "S apply", "S iFFT", "S OLA", "S peak", "A load issue",
          "A bins", "-", "-", "-"]
# the per-utterance synthesis kernel (avz_synthesis_utt_kernel)
UTT_PHASES = {4: "U window+FFT", 5: "U apply", 6: "U next loads", 7: "U iFFT",
              8: "U barrier 1", 9: "U OLA+rescale", 10: "U barrier 2", 13: "U load wait",
              14: "U utt end", 15: "U solve"}
RS_PHASES = {4: "P prologue", 5: "P window+FFT", 6: "P next loads", 7: "P barrier",
             8: "C apply", 9: "C iFFT", 10: "C sync wait", 13: "C OLA", 14: "C barrier",
             15: "C item coefs"}

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--n-fft", type=int, default=1024)
ap.add_argument("--mask", default="ibm")
ap.add_argument("--normalize", default="peak")
ap.add_argument("--seconds", type=float, default=4.0)
ap.add_argument("--synth-variant", type=int, default=-1, help="plan.set_diagnostics synth_variant")
ap.add_argument("--rows", default="",
                help="lo:hi[,lo:hi...] block-row groups to report separately (e.g. 0:8,8:256)")
ap.add_argument("--kappa", type=float, default=None, help="IBM plans: ibm_kappa")
ap.add_argument("--exact", action="store_true",
                help="label slots 4-10 as the exact IBM path's round phases (analysis)")
ap.add_argument("--utt", action="store_true",
                help="label slots 4-10, 13-15 as the per-utterance synthesis kernel's phases")
a = ap.parse_args()
if a.synth_variant >= 0 and not a.utt:
    PHASES = [RS_PHASES.get(i, n) if i >= 4 and a.synth_variant == 1 else n
              for i, n in enumerate(PHASES)]
if a.exact:
    PHASES = [{4: "X loads+ref A", 5: "X ref B", 6: "X barrier 1", 7: "X mic FFT",
               8: "X barrier 2", 9: "X bins", 10: "X barrier 3", 13: "X grid arrive",
               14: "X scan / rounds", 15: "X grid arrive 2"}.get(i, n)
              for i, n in enumerate(PHASES)]
if a.utt:
    PHASES = [UTT_PHASES.get(i, n) if i >= 4 and i not in (11, 12) else n
              for i, n in enumerate(PHASES)]
S = int(a.seconds * 16000)
dev = torch.device("cuda:0")
mix, tgt, itf = synth.make_batch(a.batch, n_samples=S, n_interferers=2)
plan = avz.MVDRPlan(n_fft=a.n_fft, sigma=1.0, mic_d=0.01, mask=a.mask,
                    postfilter="ibm" if a.mask == "ibm" else "none", normalize=a.normalize,
                    max_batch=a.batch, max_samples=S,
                    **({"ibm_kappa": a.kappa} if a.kappa is not None else {}))
d = [torch.from_numpy(x).to(dev) for x in (mix, tgt, itf)]
kw = dict(ref_tgt=d[1], ref_int=d[2]) if a.mask == "ibm" else {}
nblk = a.batch * -(-plan.frames(S) // avz._lib.lib.avz_chunk_frames())
st = torch.zeros((nblk, 16), dtype=torch.int64, device=dev)
lib = avz._lib.lib
if a.synth_variant >= 0:
    plan.set_diagnostics(synth_variant=a.synth_variant)

setter = lib.avz_debug_set_stamps_chunked
setter.argtypes = [ct.c_void_p]
for _ in range(3):
    plan.run(d[0], **kw)
torch.cuda.synchronize()
st.zero_()
assert setter(ct.c_void_p(st.data_ptr())) == 0
reps = 5
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    plan.run(d[0], **kw)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
us = st.double().cpu().numpy() / reps / 100.0  # 100 MHz ticks -> us
print(f"kernel {ms*1e3:.1f} us/launch (stamped build), B={a.batch}, N={a.n_fft}, mask={a.mask}")
groups = [tuple(int(v) for v in g.split(":")) for g in a.rows.split(",")] if a.rows else [None]
full = us
for g in groups:
    us = full[g[0]:g[1]] if g else full
    us = us[us.sum(axis=1) > 0]  # persistent grids: only the launched blocks' rows
    tot = us.sum(axis=1)
    if g:
        print(f"== block rows {g[0]}:{g[1]}")
    print(f"per-block stamped total: mean {tot.mean():.1f} us, min {tot.min():.1f}, "
          f"max {tot.max():.1f}")
    for i, n in enumerate(PHASES):
        print(f"  {n:10s} {us[:, i].mean():8.1f} us  {100*us[:, i].mean()/tot.mean():5.1f} %")
    if a.exact:  # the exact path runs on few blocks: its critical path is the busiest one's
        xs = us[:, 4:11].sum(axis=1)
        busy = np.argsort(-xs)[:6]
        print(f"exact-path blocks: {int((xs > 0).sum())} of {len(xs)}; busiest (slots 4-10, us):")
        for r in busy:
            print(f"  row {r}: total {tot[r]:.1f}, exact {xs[r]:.1f}: "
                  + " ".join(f"{us[r, i]:.1f}" for i in range(4, 11)))
