"""Mirror of rt_av_zoom/core/oracle_debug.py on the MI355X engine.

``main`` reads the same three WAVs from OUTDIR (oracle_debug.py:25-39), runs the
oracle-IBM MVDR chain (:42-94) in one fused HIP launch (``avz_mvdr_batch`` with
AVZ_MASK_IBM, AVZ_PF_IBM_TARGET, s /= max|s|) and writes output_oracle.wav (:96).
N_FFT/N_HOP/SIGMA are module globals exactly as in the reference, so callers can patch
them the same way.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import wavio
from .engine import MVDRPlan
from .masked_mvdr import C, D, FS, N_FFT, N_HOP, N_MICS  # noqa: F401  (oracle_debug.py:11-19)

ANGLE_TARGET = 90.0
SIGMA = 1
OUTDIR = "simulation_results/ljspeech_anechoic_20251130_154029"


def enhance(y_mix, s_tgt, s_int, n_fft=None, sigma=None, d=None, device="cuda"):
    """[2, S] mixture + two mono references -> peak-normalised output (float32 numpy)."""
    n_fft = N_FFT if n_fft is None else n_fft
    sigma = SIGMA if sigma is None else sigma
    d = D if d is None else d
    S = y_mix.shape[1]
    plan = MVDRPlan(n_fft=n_fft, sigma=float(sigma), mic_d=d, c_sound=C, angle_deg=ANGLE_TARGET,
                    mask="ibm", postfilter="ibm", normalize="peak", norm_eps=0.0,
                    max_batch=1, max_samples=S)
    dev = torch.device(device)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))[None].to(dev)  # noqa: E731
    out, _ = plan.run(t(y_mix), ref_tgt=t(s_tgt[:S]), ref_int=t(s_int[:S]))
    return out[0, :plan.out_len(S)].cpu().numpy()


def main(outdir=None):
    outdir = OUTDIR if outdir is None else outdir
    print("--- ORACLE TEST: Can the code theoretically work? ---")
    if not (os.path.exists(f"{outdir}//target_reference.wav")
            and os.path.exists(f"{outdir}//interference_reference.wav")):
        print("Error: Reference files missing. Run world.py first.")
        return None
    y_mix, _ = wavio.read(f"{outdir}//mixture.wav", dtype="float32")
    s_tgt, _ = wavio.read(f"{outdir}//target_reference.wav", dtype="float32")
    s_int, _ = wavio.read(f"{outdir}//interference_reference.wav", dtype="float32")
    s_out = enhance(y_mix.T, s_tgt, s_int, N_FFT, SIGMA, D)
    wavio.write(f"{outdir}/output_oracle.wav", s_out, FS)
    print(f"Saved '{outdir}/output_oracle.wav'.")
    return s_out
