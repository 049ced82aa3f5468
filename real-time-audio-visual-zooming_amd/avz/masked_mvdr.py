"""Mirror of rt_av_zoom/core/masked_mvdr.py on the MI355X engine.

Same module constants (masked_mvdr.py:9-18) and function names; ``main`` runs the
heuristic IPD-mask MVDR (masked_mvdr.py:50-132) through the fused HIP kernel
(``avz_mvdr_batch`` with AVZ_MASK_IPD, no post-filter, s /= max|s| + 1e-6).
The mask PNG of the reference (:84-88) is not produced.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import wavio
from .engine import MVDRPlan

FS = 16000
D = 0.01
C = 343.0
ANGLE_TARGET = 90.0
N_MICS = 2
SIGMA = 1e-7
N_FFT = 512
N_HOP = 256


def get_steering_vector(angle_deg, f, d, c):
    """masked_mvdr.py:22-35 — (2, 1) complex128 far-field steering vector (host helper;
    the kernels evaluate the same expression per bin in fp64)."""
    theta = np.deg2rad(angle_deg)
    tau1 = (d / 2) * np.cos(0.0) * np.cos(theta - 0) / c
    tau2 = (d / 2) * np.cos(0.0) * np.cos(theta - np.pi) / c
    omega = 2 * np.pi * f
    return np.array([[np.exp(-1j * omega * tau1)], [np.exp(-1j * omega * tau2)]], dtype=complex)


def compute_hard_geometric_mask(Y_stft, freqs=None):
    """masked_mvdr.py:37-46 on the device: 1.0 where angle(Y0) != angle(Y1), else 0.01.
    Y_stft: [C, F, T] complex64 (torch device tensor or numpy, moved to cuda)."""
    Y = Y_stft if isinstance(Y_stft, torch.Tensor) else torch.from_numpy(np.asarray(Y_stft))
    if not Y.is_cuda:
        Y = Y.cuda()
    Y = Y.to(torch.complex64)
    pd = torch.angle(Y[0]) - torch.angle(Y[1])
    one = torch.ones((), dtype=torch.float64, device=Y.device)
    return torch.where(pd.abs() > 0, one, 0.01 * one)


def enhance(y_mix: np.ndarray, n_fft=N_FFT, sigma=SIGMA, d=D, device="cuda") -> np.ndarray:
    """y_mix [2, S] float32 -> peak-normalised beamformed waveform (float32 numpy)."""
    S = y_mix.shape[1]
    plan = MVDRPlan(n_fft=n_fft, sigma=sigma, mic_d=d, c_sound=C, angle_deg=ANGLE_TARGET,
                    mask="ipd", postfilter="none", normalize="peak", norm_eps=1e-6,
                    max_batch=1, max_samples=S)
    mix = torch.from_numpy(np.ascontiguousarray(y_mix, dtype=np.float32))[None].to(device)
    out, _ = plan.run(mix)
    return out[0, :plan.out_len(S)].cpu().numpy()


def main(output_dir_world):
    """masked_mvdr.py:50-135: <dir>/mixture_3_sources.wav -> ../MVDR_Outputs/output_masked_mvdr.wav"""
    if not output_dir_world or not os.path.exists(output_dir_world):
        print(f"ERROR: Invalid directory provided: {output_dir_world}")
        return None
    input_file = os.path.join(output_dir_world, "mixture_3_sources.wav")
    if not os.path.exists(input_file):
        print(f"Error: {input_file} not found.")
        return None
    out_dir = os.path.join(os.path.dirname(output_dir_world), "MVDR_Outputs")
    os.makedirs(out_dir, exist_ok=True)
    y, fs = wavio.read(input_file, dtype="float32")
    s_out = enhance(y.T, N_FFT, SIGMA, D)
    path = os.path.join(out_dir, "output_masked_mvdr.wav")
    wavio.write(path, s_out, fs)
    print(f"Saved outputs to: {out_dir}")
    return s_out
