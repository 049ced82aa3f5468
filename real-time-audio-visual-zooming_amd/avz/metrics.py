"""Projection SIR / SDR / OSINR and the evaluation report formats.

Semantics: scripts/run_metrics.py:6-36 (calculate_metrics_manual: all three signals
unit-normalised, SIR = 10 log10(alpha^2 / (beta^2 + 1e-10))) and
Final_pipeline/src/metrics.py:102-123 (calculate_osnr_osir: output NOT normalised,
OSIR = 10 log10(P_t / (P_i + eps)), OSINR with the residual). Inputs are [B, L] tensors
already aligned to a common length (the reference aligns to the minimum length,
metrics.py:91-98 / run_metrics.py:68-73); ``lengths`` masks ragged rows.

Device tensors go through the HIP kernel ``avz_projection_metrics`` (six fp64 inner
products per utterance in one streaming pass, then the reference's formulas). Host
tensors (CPU-only tooling and the gloo tests) use the same formulas in torch fp64.

``evaluate_run`` mirrors metrics.py:125-214: report.txt (same lines) and the
batch_metrics.csv row; STOI/PESQ are 0.0 exactly as the reference writes them when
pystoi/pesq are missing (metrics.py:8-14), which is the case in this image.
"""
from __future__ import annotations

import csv
import ctypes as ct
import datetime
import os

import numpy as np
import torch

EPS = 1e-10
CSV_HEADER = ["Run_ID", "SIR_Base", "SIR_Enh", "SIR_Imp", "SINR_Base", "SINR_Enh", "STOI",
              "PESQ_WB", "PESQ_NB"]


# ----------------------------------------------------------------------------- device path
def projection_metrics(est: torch.Tensor, tgt: torch.Tensor, itf: torch.Tensor, lengths=None,
                       stream=None, est_peak: torch.Tensor | None = None, est_eps: float = 0.0):
    """HIP: -> float64 [B, 4] = (OSINR, OSIR, SDR, SIR) per row, in dB. With ``est_peak``
    the rows are scored as est / (est_peak + est_eps) (an un-normalised output and its
    peak, as a NORM_NONE plan returns them), the scale applied inside the fp64 sums."""
    from ._lib import check, lib
    from .engine import _stream_handle
    est, tgt, itf = (x.float().contiguous() if x.dtype != torch.float32 or x.stride(-1) != 1
                     else x for x in (est, tgt, itf))
    if est.dim() == 1:
        est, tgt, itf = est[None], tgt[None], itf[None]
    B, L = est.shape
    dev = est.device
    if lengths is None:
        lengths = torch.full((B,), L, dtype=torch.int32, device=dev)
    else:
        lengths = torch.as_tensor(lengths, dtype=torch.int32).to(dev)
    sums = torch.empty((B, 6), dtype=torch.float64, device=dev)
    out = torch.empty((B, 4), dtype=torch.float64, device=dev)
    p = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    if est_peak is not None:
        pk = est_peak.float().contiguous()
        assert pk.numel() == B and pk.device == dev
        check(lib.avz_projection_metrics_scaled(B, L, p(lengths), p(est), est.stride(0), p(pk),
                                                float(est_eps), p(tgt), tgt.stride(0), p(itf),
                                                itf.stride(0), p(sums), p(out),
                                                _stream_handle(stream)),
              "avz_projection_metrics_scaled")
        return out
    check(lib.avz_projection_metrics(B, L, p(lengths), p(est), est.stride(0), p(tgt),
                                     tgt.stride(0), p(itf), itf.stride(0), p(sums), p(out),
                                     _stream_handle(stream)), "avz_projection_metrics")
    return out


# ----------------------------------------------------------------------------- host path
def _masked(x: torch.Tensor, lengths):
    x = x.double()
    if lengths is None:
        return x
    idx = torch.arange(x.shape[-1], device=x.device)
    return x * (idx[None, :] < torch.as_tensor(lengths, device=x.device)[:, None]).double()


def _host_manual(output, target, interf, lengths=None):
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


def _host_osnr_osir(output, target, interf, lengths=None):
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


def calculate_metrics_manual(output, target, interf, lengths=None):
    """Batched run_metrics.calculate_metrics_manual -> (sdr [B], sir [B]) in dB."""
    if output.is_cuda:
        m = projection_metrics(output, target, interf, lengths)
        return m[:, 2], m[:, 3]
    return _host_manual(output, target, interf, lengths)


def calculate_osnr_osir(output, target, interf, lengths=None, peak=None, eps=0.0):
    """Batched Final_pipeline/src/metrics.calculate_osnr_osir -> (osinr [B], osir [B]).
    ``peak``: score output / (peak + eps) (an un-normalised output and its peak)."""
    if output.is_cuda:
        m = projection_metrics(output, target, interf, lengths, est_peak=peak, est_eps=eps)
        return m[:, 0], m[:, 1]
    if peak is not None:
        output = output.double() / (peak.double()[:, None] + eps)
    return _host_osnr_osir(output, target, interf, lengths)


# ----------------------------------------------------------------------------- reports
def load_and_align(sim_dir, result_path):
    """metrics.py:70-99: channel 0 of each file, aligned to the minimum length."""
    from . import wavio
    try:
        s_est, _ = wavio.read(result_path, dtype="float32")
        s_tgt, _ = wavio.read(os.path.join(sim_dir, "target.wav"), dtype="float32")
        s_int, _ = wavio.read(os.path.join(sim_dir, "interference.wav"), dtype="float32")
        s_mix, _ = wavio.read(os.path.join(sim_dir, "mixture.wav"), dtype="float32")
    except FileNotFoundError as e:
        print(f"[EVAL] Error: Missing file - {e}")
        return None, None, None, None
    s_mix, s_est, s_tgt, s_int = (x[:, 0] if x.ndim > 1 else x
                                  for x in (s_mix, s_est, s_tgt, s_int))
    n = min(len(s_est), len(s_tgt), len(s_int), len(s_mix))
    return s_est[:n], s_tgt[:n], s_int[:n], s_mix[:n]


def format_report(run_name, m, timestamp=None):
    """report.txt lines of metrics.py:166-182 for m = dict(sir_b, sinr_b, sir_s, sinr_s,
    stoi, pesq_wb, pesq_nb)."""
    ts = timestamp or datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S")
    imp = m["sir_s"] - m["sir_b"]
    return "\n".join([
        f"=== EVALUATION REPORT: {run_name} ===",
        f"Date: {ts}",
        "------------------------------------",
        "BASELINE (Mixture):",
        f"  SIR:   {m['sir_b']:.2f} dB",
        f"  SINR:  {m['sinr_b']:.2f} dB",
        "------------------------------------",
        "ENHANCED (Output):",
        f"  SIR:   {m['sir_s']:.2f} dB",
        f"  SINR:  {m['sinr_s']:.2f} dB",
        f"  STOI:  {m['stoi']:.4f}",
        f"  PESQ:  {m['pesq_wb']:.4f} (WB) | {m['pesq_nb']:.4f} (NB)",
        "------------------------------------",
        f"SIR IMPROVEMENT: {imp:+.2f} dB",
        "===================================="])


def csv_row(run_name, m):
    """One batch_metrics.csv row (metrics.py:16-44)."""
    return {"Run_ID": run_name, "SIR_Base": f"{m['sir_b']:.2f}", "SIR_Enh": f"{m['sir_s']:.2f}",
            "SIR_Imp": f"{m['sir_s'] - m['sir_b']:.2f}", "SINR_Base": f"{m['sinr_b']:.2f}",
            "SINR_Enh": f"{m['sinr_s']:.2f}", "STOI": f"{m['stoi']:.4f}",
            "PESQ_WB": f"{m['pesq_wb']:.4f}", "PESQ_NB": f"{m['pesq_nb']:.4f}"}


def append_to_csv(csv_path, rows):
    new = not os.path.isfile(csv_path)
    with open(csv_path, "a", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=CSV_HEADER)
        if new:
            w.writeheader()
        w.writerows(rows)


def evaluate_run(run_name, sim_dir_root=os.path.join("data", "simulated"),
                 results_dir=os.path.join("data", "results"), device=None):
    """metrics.py:125-214 on the device: OSIR/OSINR of the mixture (baseline) and of the
    enhanced output in one avz_projection_metrics call; writes report.txt and appends
    the batch_metrics.csv row. Returns the metrics dict."""
    sim_dir = os.path.join(sim_dir_root, run_name)
    res_dir = os.path.join(results_dir, f"{run_name}_results")
    est_path = os.path.join(res_dir, f"{run_name}_enhanced.wav")
    if not os.path.exists(est_path):
        print(f"[EVAL] Error: Inference output not found at {est_path}")
        return None
    print(f"[EVAL] Evaluating: {run_name}...")
    s_est, s_tgt, s_int, s_mix = load_and_align(sim_dir, est_path)
    if s_est is None:
        return None
    dev = device or torch.device("cuda", torch.cuda.current_device())
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    est = torch.stack([t(s_mix), t(s_est)])
    tg = t(s_tgt)[None].expand(2, -1).contiguous()
    it = t(s_int)[None].expand(2, -1).contiguous()
    mm = projection_metrics(est, tg, it).cpu().numpy()
    m = dict(sir_b=float(mm[0, 1]), sinr_b=float(mm[0, 0]), sir_s=float(mm[1, 1]),
             sinr_s=float(mm[1, 0]), stoi=0.0, pesq_wb=0.0, pesq_nb=0.0)
    report = format_report(run_name, m)
    print(report)
    with open(os.path.join(res_dir, "report.txt"), "w") as fh:
        fh.write(report)
    print(f"[EVAL] Report saved to: {os.path.join(res_dir, 'report.txt')}")
    append_to_csv(os.path.join(results_dir, "batch_metrics.csv"), [csv_row(run_name, m)])
    return m
