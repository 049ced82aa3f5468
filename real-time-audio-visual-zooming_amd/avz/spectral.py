"""Spectral-domain operator surface: drop-ins for the reference's functions that take an
STFT, backed by ``avz_beamform_spectral`` / ``avz_istft`` (include/avz.h).

* ``get_all_steering_vectors(f_bins, angle_deg, d, c)`` —
  rt_av_zoom/core/tf_lite_version/inference.py:53-81 (host table, [F, 2, 1] complex128).
* ``batch_mvdr(Y, mask, f_bins, d_vectors, sigma)`` — tf_lite_version/inference.py:85-179:
  numpy in, numpy out ([F, T] complex128), the item-level LinAlgError fallback included.
* ``hybrid_hard_null_bf(Y, mask, f_bins)`` — Final_pipeline/src/inference.py:28-98.
* ``SpectralBeamformer`` — the batched device form: Y [B, 2, F, T] complex64 and masks
  [B, F, T] resident in HBM -> S [B, F, T] (post-filter fused) -> iSTFT.

The numpy-facing functions copy to and from the device (PCIe); callers with device
tensors use ``SpectralBeamformer`` / ``MVDRPlan.beamform_spectral`` directly. There is no
CPU fallback: every function runs the HIP kernels.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import MVDRPlan

FS = 16000
ANGLE_TARGET = 90.0
SIGMA_TFLITE = 1e-5       # tf_lite_version/inference.py:46
D_TFLITE = 0.04           # tf_lite_version/config.json "d"
D_FINAL = 0.08            # Final_pipeline/src/config.py:29 (MIC_DIST)
C_SOUND = 343.0


def get_all_steering_vectors(f_bins, angle_deg: float, d: float, c: float) -> np.ndarray:
    """tf_lite_version/inference.py:53-81: [F, 2, 1] complex128 far-field steering vectors."""
    th = np.deg2rad(angle_deg)
    om = 2 * np.pi * np.asarray(f_bins, dtype=np.float64)
    sv = np.stack([np.exp(-1j * om * ((d / 2) * np.cos(th) / c)),
                   np.exp(-1j * om * ((d / 2) * np.cos(th - np.pi) / c))], axis=0)
    return np.expand_dims(sv.T, axis=-1)


def _n_fft_of(F: int) -> int:
    n = 2 * (F - 1)
    if n not in (512, 1024):
        raise ValueError(f"{F} bins: only n_fft 512 / 1024 spectra are supported")
    return n


def _check_bins(f_bins, n_fft: int, fs: int):
    f = np.asarray(f_bins, dtype=np.float64)
    if f.shape != (n_fft // 2 + 1,) or np.abs(f - np.fft.rfftfreq(n_fft, 1.0 / fs)).max() > 1e-6:
        raise ValueError("f_bins must be the rfft bin frequencies of the spectrum")


_PLANS: dict = {}


def _plan(kind: str, n_fft: int, sigma: float, batch: int, d: float, floor=None,
          device=None) -> MVDRPlan:
    key = (kind, n_fft, float(sigma), batch, float(d), floor, str(device))
    p = _PLANS.get(key)
    if p is None:
        pf = "none" if floor is None else ("floor" if floor > 0 else "mul")
        if kind == "mvdr":  # batch_mvdr semantics (include/avz.h, avz_beamform_spectral)
            p = MVDRPlan(n_fft=n_fft, fs=FS, sigma=sigma, mic_d=d, mask="external", postfilter=pf,
                         pf_floor=floor or 0.0, weight_eps=1e-10, fmin_hz=0.0,
                         singular_fallback="batch", normalize="none", max_batch=batch,
                         max_samples=n_fft)
        else:  # hybrid_hard_null_bf
            p = MVDRPlan(n_fft=n_fft, fs=FS, mic_d=d, mask="external", postfilter=pf,
                         pf_floor=floor or 0.0, beamformer="hybrid_null", bypass_hz=200.0,
                         cond_max=10.0, normalize="none", max_batch=batch, max_samples=n_fft)
        _PLANS[key] = p
    return p


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("avz.spectral needs the HIP device (there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def batch_mvdr(Y, mask, f_bins, d_vectors, sigma) -> np.ndarray:
    """tf_lite_version/inference.py:85-179 on the device: Y [2, F, T] complex, mask [F, T]
    target probability, d_vectors [F, 2, 1] (get_all_steering_vectors), sigma -> S [F, T]
    complex128 (computed in fp64/fp32 on the device, returned in the reference's dtype)."""
    Y = np.asarray(Y)
    F, T = Y.shape[1], Y.shape[2]
    n_fft = _n_fft_of(F)
    dev = _device()
    plan = _plan("mvdr", n_fft, sigma, 1, D_TFLITE, device=dev)
    dY = torch.from_numpy(np.ascontiguousarray(Y, dtype=np.complex64))[None].to(dev)
    dM = torch.from_numpy(np.ascontiguousarray(mask, dtype=np.float32))[None].to(dev)
    st = torch.from_numpy(np.ascontiguousarray(np.asarray(d_vectors)[:, :, 0],
                                               dtype=np.complex128)).to(dev)
    S = plan.beamform_spectral(dY, dM, steer=st)
    return S[0].cpu().numpy().astype(np.complex128)


def hybrid_hard_null_bf(Y, mask, f_bins, d: float = D_FINAL) -> np.ndarray:
    """Final_pipeline/src/inference.py:28-98 on the device: Y [2, F, T], mask [F, T] target
    probability, f_bins (rfft frequencies) -> S [F, T] complex128."""
    Y = np.asarray(Y)
    n_fft = _n_fft_of(Y.shape[1])
    _check_bins(f_bins, n_fft, FS)
    dev = _device()
    plan = _plan("hybrid", n_fft, 0.0, 1, d, device=dev)
    dY = torch.from_numpy(np.ascontiguousarray(Y, dtype=np.complex64))[None].to(dev)
    dM = torch.from_numpy(np.ascontiguousarray(mask, dtype=np.float32))[None].to(dev)
    S = plan.beamform_spectral(dY, dM)
    return S[0].cpu().numpy().astype(np.complex128)


class SpectralBeamformer:
    """Batched device form of batch_mvdr / hybrid_hard_null_bf with the chunk drivers'
    post-filters fused (max_frames: the longest spectra istft() will see; 64 = a 2-s chunk) (tf_lite_version/inference.py:350 S * max(M, 0.05);
    Final_pipeline/src/inference.py:219 S * M) and the iSTFT of the result.

    kind "mvdr" (sigma 1e-5, d 0.04, floor 0.05 by default) or "hybrid" (d 0.08, x M)."""

    def __init__(self, kind: str = "mvdr", n_fft: int = 1024, max_items: int = 1,
                 sigma: float = SIGMA_TFLITE, d: float | None = None, floor: float | None = 0.05,
                 max_frames: int = 64):
        if kind not in ("mvdr", "hybrid"):
            raise ValueError("kind must be 'mvdr' or 'hybrid'")
        d = (D_TFLITE if kind == "mvdr" else D_FINAL) if d is None else d
        pf = "none" if floor is None else ("floor" if (kind == "mvdr" and floor > 0) else "mul")
        common = dict(n_fft=n_fft, fs=FS, mic_d=d, mask="external", postfilter=pf,
                      pf_floor=floor or 0.0, normalize="none", max_batch=max_items,
                      max_samples=max((max_frames - 1) * (n_fft // 2), n_fft))
        if kind == "mvdr":
            self.plan = MVDRPlan(sigma=sigma, weight_eps=1e-10, fmin_hz=0.0,
                                 singular_fallback="batch", **common)
        else:
            self.plan = MVDRPlan(beamformer="hybrid_null", bypass_hz=200.0, cond_max=10.0,
                                 **common)

    def beamform(self, Y: torch.Tensor, mask: torch.Tensor, **kw) -> torch.Tensor:
        return self.plan.beamform_spectral(Y, mask, **kw)

    def istft(self, S: torch.Tensor, **kw):
        return self.plan.istft(S, **kw)
