"""Projection SIR / SDR / OSINR on the device, batched.

Semantics follow scripts/run_metrics.py:6-36 (calculate_metrics_manual: all three
signals unit-normalised, SIR = 10 log10(alpha^2 / (beta^2 + 1e-10))) and
Final_pipeline/src/metrics.py:102-123 (calculate_osnr_osir: output NOT normalised,
OSIR = 10 log10(P_t / (P_i + eps)), OSINR with the residual). Inputs are [B, L] tensors
already aligned to a common length (the reference aligns to the minimum length,
metrics.py:91-98 / run_metrics.py:68-73); ``lengths`` masks ragged rows. Reductions
run in float64 on whichever device the tensors live on.
"""
from __future__ import annotations

import torch

EPS = 1e-10


def _masked(x: torch.Tensor, lengths):
    x = x.double()
    if lengths is None:
        return x
    idx = torch.arange(x.shape[-1], device=x.device)
    return x * (idx[None, :] < lengths[:, None]).double()


def calculate_metrics_manual(output, target, interf, lengths=None):
    """Batched run_metrics.calculate_metrics_manual -> (sdr [B], sir [B]) in dB."""
    o, t, i = (_masked(v, lengths) for v in (output, target, interf))
    o = o / (o.norm(dim=-1, keepdim=True) + EPS)
    t = t / (t.norm(dim=-1, keepdim=True) + EPS)
    i = i / (i.norm(dim=-1, keepdim=True) + EPS)
    a = (o * t).sum(-1, keepdim=True)
    b = (o * i).sum(-1, keepdim=True)
    e_t, e_i = a * t, b * i
    e_a = o - e_t - e_i
    p_t = (e_t ** 2).sum(-1)
    p_i = (e_i ** 2).sum(-1) + 1e-10
    p_n = (e_a ** 2).sum(-1) + 1e-10
    return 10 * torch.log10(p_t / (p_i + p_n)), 10 * torch.log10(p_t / p_i)


def calculate_osnr_osir(output, target, interf, lengths=None):
    """Batched Final_pipeline/src/metrics.calculate_osnr_osir -> (osinr [B], osir [B])."""
    o, t, i = (_masked(v, lengths) for v in (output, target, interf))
    t = t / (t.norm(dim=-1, keepdim=True) + EPS)
    i = i / (i.norm(dim=-1, keepdim=True) + EPS)
    a = (o * t).sum(-1, keepdim=True)
    b = (o * i).sum(-1, keepdim=True)
    e_t, e_i = a * t, b * i
    e_n = o - e_t - e_i
    p_t = (e_t ** 2).sum(-1)
    p_i = (e_i ** 2).sum(-1)
    p_n = (e_n ** 2).sum(-1)
    return 10 * torch.log10(p_t / (p_i + p_n + EPS)), 10 * torch.log10(p_t / (p_i + EPS))
