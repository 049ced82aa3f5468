"""Mirror of rt_av_zoom/core/oracle_reverb.py on the MI355X engine.

``main(args)`` reads ``mixture_wpe.wav`` + the two references from ``args.outdir``
(oracle_reverb.py:50-71), runs the oracle-IBM MVDR chain with the experiment hooks
``args.sigma`` (diagonal loading, :124) and ``args.hp`` (high-pass cutoff, :116) and the
ideal-ratio-mask post-filter (:143-156) in one ``avz_mvdr_batch`` call
(AVZ_MASK_IBM + AVZ_PF_IRM, singular bins -> ones/2 as :133-135, s /= max|s| + 1e-9 as
:164) and writes ``output_oracle_reverb.wav`` (:170-172). Producing mixture_wpe.wav
(WPE dereverberation, rt_av_zoom/core/dereverb.py) is out of scope.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from . import wavio
from .engine import MVDRPlan
from .masked_mvdr import C, D, FS, N_FFT, N_HOP, N_MICS  # noqa: F401  (oracle_reverb.py:25-29)

ANGLE_TARGET = 90.0
DEFAULT_OUTDIR = "simulation_results/ljspeech_reverb_20251130_215709"


def enhance(y_mix, s_tgt, s_int, sigma=1e-3, hp_cutoff=100.0, n_fft=None, d=None,
            device="cuda"):
    """[2, S] mixture + two mono references -> normalised output (float32 numpy)."""
    n_fft = N_FFT if n_fft is None else n_fft
    d = D if d is None else d
    S = y_mix.shape[1]
    plan = MVDRPlan(n_fft=n_fft, sigma=float(sigma), fmin_hz=float(hp_cutoff), mic_d=d,
                    c_sound=C, angle_deg=ANGLE_TARGET, mask="ibm", postfilter="irm",
                    singular_fallback="mean", normalize="peak", norm_eps=1e-9,
                    max_batch=1, max_samples=S)
    dev = torch.device(device)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))[None].to(dev)  # noqa: E731
    out, _ = plan.run(t(y_mix), ref_tgt=t(s_tgt[:S]), ref_int=t(s_int[:S]))
    return out[0, :plan.out_len(S)].cpu().numpy()


def main(args):
    outdir, sigma, hp_cutoff = args.outdir, args.sigma, args.hp
    print("\n--- ORACLE OPTIMIZATION RUN ---")
    print(f"Directory:  {os.path.basename(outdir)}")
    print(f"Parameters: Sigma={sigma} | HP_Cutoff={hp_cutoff} Hz")
    if not os.path.exists(outdir):
        print(f"ERROR: Directory not found: {outdir}")
        return None
    path_mix = os.path.join(outdir, "mixture_wpe.wav")
    path_tgt = os.path.join(outdir, "target_reference.wav")
    path_int = os.path.join(outdir, "interference_reference.wav")
    if not (os.path.exists(path_mix) and os.path.exists(path_tgt) and os.path.exists(path_int)):
        print("CRITICAL ERROR: Audio files missing (mixture/target/interference).")
        return None
    y_mix, _ = wavio.read(path_mix, dtype="float32")
    if y_mix.ndim > 1 and y_mix.shape[0] > y_mix.shape[1]:  # (:64-65) to (channels, samples)
        y_mix = y_mix.T
    s_tgt, _ = wavio.read(path_tgt, dtype="float32")
    s_int, _ = wavio.read(path_int, dtype="float32")
    s_out = enhance(y_mix, s_tgt, s_int, sigma, hp_cutoff)
    out_path = os.path.join(outdir, "output_oracle_reverb.wav")
    wavio.write(out_path, s_out, FS)
    print(f"Saved: {out_path}")
    return s_out


def parse_args(argv=None):
    """The reference CLI (oracle_reverb.py:177-190)."""
    p = argparse.ArgumentParser(description="Run Optimized Oracle MVDR")
    p.add_argument("--outdir", type=str, default=DEFAULT_OUTDIR)
    p.add_argument("--sigma", type=float, default=1e-3)
    p.add_argument("--hp", type=float, default=100.0)
    return p.parse_args(argv)


if __name__ == "__main__":
    main(parse_args())
