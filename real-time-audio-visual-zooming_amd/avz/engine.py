"""Host-side plan objects over the C ABI (device memory and streams from PyTorch-ROCm).

``MVDRPlan`` is the batched form of the reference's per-utterance chain
(rt_av_zoom/core/oracle_debug.py:42-94, rt_av_zoom/core/masked_mvdr.py:76-128,
rt_av_zoom/core/full_audio_generating_pipeline/inference.py:88-118): one call runs
STFT -> mask -> masked covariance -> MVDR -> apply/post-filter -> iSTFT (-> peak
normalisation) for a whole batch of utterances in one chain of kernel launches (analysis, solve, synthesis, finalize).
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass, field

import torch

from . import _lib
from ._lib import AvzBatchArgs, AvzConfig, check, lib

MASKS = {"ibm": _lib.MASK_IBM, "ipd": _lib.MASK_IPD, "external": _lib.MASK_EXTERNAL,
         "ones": _lib.MASK_ONES}
POSTFILTERS = {"none": _lib.PF_NONE, "ibm": _lib.PF_IBM_TARGET, "floor": _lib.PF_EXT_FLOOR,
               "mul": _lib.PF_EXT_MUL, "irm": _lib.PF_IRM}
FALLBACKS = {"mic0": _lib.FALLBACK_MIC0, "mean": _lib.FALLBACK_MEAN}
NORMS = {"none": _lib.NORM_NONE, "peak": _lib.NORM_PEAK}
BEAMFORMERS = {"mvdr": _lib.BF_MVDR, "hybrid_null": _lib.BF_HYBRID_NULL}


def n_frames(length: int, hop: int) -> int:
    """scipy.signal.stft frame count with boundary='zeros', padded=True."""
    return -(-length // hop) + 1


def out_length(length: int, hop: int) -> int:
    """scipy.signal.istft output length for an utterance of ``length`` samples."""
    return (n_frames(length, hop) - 1) * hop


@dataclass
class PlanConfig:
    n_fft: int = 1024
    fs: int = 16000
    sigma: float = 1.0
    angle_deg: float = 90.0
    mic_d: float = 0.01
    c_sound: float = 343.0
    fmin_hz: float = 100.0
    mask: str = "ibm"
    postfilter: str = "ibm"
    pf_floor: float = 0.05
    weight_eps: float = 0.0
    normalize: str = "peak"
    norm_eps: float = 0.0
    max_batch: int = 1
    max_samples: int = 64000
    beamformer: str = "mvdr"
    bypass_hz: float = 200.0
    cond_max: float = 10.0
    singular_fallback: str = "mic0"
    extra: dict = field(default_factory=dict)


def _ptr(t):
    return None if t is None else ct.c_void_p(t.data_ptr())


def _stream_handle(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ct.c_void_p(s.cuda_stream)


class MVDRPlan:
    """Immutable engine configuration + device workspace (libavz plan)."""

    def __init__(self, cfg: PlanConfig | None = None, **kw):
        cfg = cfg or PlanConfig()
        for k, v in kw.items():
            if not hasattr(cfg, k):
                raise TypeError(f"unknown plan option {k!r}")
            setattr(cfg, k, v)
        self.cfg = cfg
        c = AvzConfig()
        c.fs, c.n_fft, c.hop = cfg.fs, cfg.n_fft, cfg.n_fft // 2
        c.sigma, c.angle_deg, c.mic_d = cfg.sigma, cfg.angle_deg, cfg.mic_d
        c.c_sound, c.fmin_hz = cfg.c_sound, cfg.fmin_hz
        c.mask_mode = MASKS[cfg.mask]
        c.postfilter = POSTFILTERS[cfg.postfilter]
        c.pf_floor, c.weight_eps = cfg.pf_floor, cfg.weight_eps
        c.normalize, c.norm_eps = NORMS[cfg.normalize], cfg.norm_eps
        c.max_batch, c.max_samples = cfg.max_batch, cfg.max_samples
        c.beamformer = BEAMFORMERS[cfg.beamformer]
        c.bypass_hz, c.cond_max = cfg.bypass_hz, cfg.cond_max
        c.singular_fallback = FALLBACKS[cfg.singular_fallback]
        h = ct.c_void_p()
        check(lib.avz_plan_create(ct.byref(h), ct.byref(c)), "avz_plan_create")
        self._h = h
        self.hop = cfg.n_fft // 2
        self.F = cfg.n_fft // 2 + 1

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.avz_plan_destroy(h)
            self._h = None

    # ------------------------------------------------------------------ diagnostics
    KERNELS = ("analysis", "solve", "synthesis", "finalize")

    def set_timing(self, enable: bool = True, analysis_only: bool = False) -> None:
        """Record HIP events around each of the chain's four kernels on every run()
        (analysis_only: around the analysis kernel alone, two events per run)."""
        mode = (2 if analysis_only else 1) if enable else 0
        check(lib.avz_plan_set_timing(self._h, mode), "avz_plan_set_timing")

    def timing(self) -> dict:
        """Average ms per kernel over the runs since set_timing(True) (waits for them;
        NaN for kernels not timed)."""
        ms = (ct.c_double * 4)()
        n = ct.c_int()
        check(lib.avz_plan_get_timing(self._h, ms, ct.byref(n)), "avz_plan_get_timing")
        return {"calls": n.value, **{k: ms[i] for i, k in enumerate(self.KERNELS)}}

    # ------------------------------------------------------------------ helpers
    def frames(self, length: int) -> int:
        return check(lib.avz_num_frames(self._h, int(length)), "avz_num_frames")

    def out_len(self, length: int) -> int:
        return out_length(length, self.hop)

    def alloc_out(self, batch: int, max_len: int, device) -> torch.Tensor:
        n = self.out_len(max_len)
        return torch.empty((batch, (n + 3) // 4 * 4), dtype=torch.float32, device=device)

    # ------------------------------------------------------------------ batch call
    def workspace_bytes(self, batch: int, max_len: int) -> int:
        """Device bytes of a per-call workspace (avz_mvdr_workspace_bytes)."""
        return check(lib.avz_mvdr_workspace_bytes(self._h, int(batch), int(max_len)),
                     "avz_mvdr_workspace_bytes")

    def alloc_workspace(self, batch: int, max_len: int, device) -> torch.Tensor:
        """A per-call workspace: calls given distinct workspaces may overlap on different
        streams (include/avz.h); calls without one share the plan's and must not."""
        n = self.workspace_bytes(batch, max_len)
        return torch.empty((max(n, 1) + 255) // 256 * 256, dtype=torch.uint8, device=device)

    def run(self, mix: torch.Tensor, lengths: torch.Tensor | None = None, *,
            max_len: int | None = None, ref_tgt=None, ref_int=None, ext_mask=None,
            out: torch.Tensor | None = None, peak: torch.Tensor | None = None,
            cov_out=None, w_out=None, workspace: torch.Tensor | None = None, stream=None):
        """mix: [B, 2, S] float32 (device); lengths: [B] int32 (device, default S).
        ref_tgt/ref_int: [B, S] (IBM); ext_mask: [B, F, T] target probability (EXTERNAL).
        workspace: optional uint8 device tensor of >= workspace_bytes(B, max_len) bytes.
        Returns (out [B, >= out_len], peak [B])."""
        if not mix.is_cuda:
            raise ValueError("mix must be a device tensor")
        if mix.dtype != torch.float32 or mix.dim() != 3 or mix.shape[1] != 2:
            raise ValueError("mix must be float32 [B, 2, S]")
        if mix.stride(2) != 1:
            raise ValueError("mix must be contiguous along samples")
        B, _, S = mix.shape
        dev = mix.device
        if lengths is None:
            lengths = torch.full((B,), S, dtype=torch.int32, device=dev)
            max_len = S
        if lengths.dtype != torch.int32 or not lengths.is_cuda or lengths.dim() != 1 \
                or lengths.shape[0] < B:
            raise ValueError("lengths must be an int32 device tensor of >= B entries")
        if max_len is None:
            max_len = int(lengths[:B].max().item())
        if max_len > S:
            raise ValueError(f"max_len {max_len} exceeds the {S} samples of mix")
        T = self.frames(max_len)
        if out is None:
            out = self.alloc_out(B, max_len, dev)
        if peak is None:
            peak = torch.empty((B,), dtype=torch.float32, device=dev)
        if out.dtype != torch.float32 or out.dim() != 2 or out.shape[0] < B or \
                out.shape[1] < self.out_len(max_len) or out.stride(1) != 1:
            raise ValueError("out must be float32 [>= B, >= out_len(max_len)]")
        if peak.dtype != torch.float32 or peak.numel() < B or not peak.is_contiguous():
            raise ValueError("peak must be a contiguous float32 tensor of >= B entries")
        a = AvzBatchArgs()
        a.batch = B
        a.len = lengths.data_ptr()
        a.max_len = int(max_len)
        a.mix = mix.data_ptr()
        a.mix_stride = mix.stride(0)
        a.ch_stride = mix.stride(1)
        for r in (ref_tgt, ref_int):
            if r is not None and (r.dtype != torch.float32 or r.stride(-1) != 1 or not r.is_cuda
                                  or r.dim() != 2 or r.shape[0] < B or r.shape[1] < max_len):
                raise ValueError("references must be float32 device tensors [B, >= max_len]")
        if ref_tgt is not None:
            a.ref_tgt = ref_tgt.data_ptr()
            a.ref_stride = ref_tgt.stride(0)
        if ref_int is not None:
            a.ref_int = ref_int.data_ptr()
            if ref_tgt is not None and ref_int.stride(0) != ref_tgt.stride(0):
                raise ValueError("ref_tgt and ref_int must share a stride")
        if ext_mask is not None:
            if ext_mask.dtype != torch.float32 or not ext_mask.is_cuda or ext_mask.dim() != 3:
                raise ValueError("ext_mask must be float32 [B, F, T] on the device")
            if ext_mask.shape[0] < B or ext_mask.shape[1] < self.F or ext_mask.shape[2] < T:
                raise ValueError(f"ext_mask {tuple(ext_mask.shape)} does not cover "
                                 f"[B={B}, F={self.F}, T={T}]")
            a.ext_mask = ext_mask.data_ptr()
            a.mask_stride_b, a.mask_stride_f, a.mask_stride_t = ext_mask.stride()
            a.mask_bins, a.mask_frames = ext_mask.shape[1], ext_mask.shape[2]
        a.out = out.data_ptr()
        a.out_stride = out.stride(0)
        a.peak = peak.data_ptr()
        a.cov_out = 0 if cov_out is None else cov_out.data_ptr()
        a.w_out = 0 if w_out is None else w_out.data_ptr()
        if workspace is not None:
            if workspace.dtype != torch.uint8 or not workspace.is_cuda:
                raise ValueError("workspace must be a uint8 device tensor")
            a.workspace = workspace.data_ptr()
            a.workspace_bytes = workspace.numel()
        check(lib.avz_mvdr_batch(self._h, ct.byref(a), _stream_handle(stream)), "avz_mvdr_batch")
        return out, peak

    def stft(self, x: torch.Tensor, lengths: torch.Tensor | None = None, max_len=None,
             stream=None) -> torch.Tensor:
        """scipy.signal.stft(x, fs, nperseg=n_fft, noverlap=n_fft//2) for x [B, C, S]
        (C in {1, 2}); returns complex64 [B, C, F, T]."""
        if x.dim() != 3 or x.dtype != torch.float32 or x.stride(2) != 1 or not x.is_cuda:
            raise ValueError("x must be float32 [B, C, S] on the device")
        B, Cn, S = x.shape
        if lengths is None:
            lengths = torch.full((B,), S, dtype=torch.int32, device=x.device)
            max_len = S
        if max_len is None:
            max_len = int(lengths.max().item())
        T = n_frames(max_len, self.hop)
        Y = torch.zeros((B, Cn, self.F, T), dtype=torch.complex64, device=x.device)
        check(lib.avz_stft(self._h, B, Cn, ct.c_void_p(lengths.data_ptr()), int(max_len),
                           ct.c_void_p(x.data_ptr()), x.stride(0), x.stride(1),
                           ct.c_void_p(Y.data_ptr()), Y.stride(0), Y.stride(1), Y.stride(2),
                           _stream_handle(stream)), "avz_stft")
        return Y


FEATURE_LAYOUTS = {"unet": _lib.FEAT_LOGMAG_IPD, "tflite": _lib.FEAT_TFLITE}


def mask_features(plan: MVDRPlan, x: torch.Tensor, layout: str = "unet", lengths=None,
                  max_len=None, stream=None) -> torch.Tensor:
    """Mask-model input features of a [B, 2, S] mic pair (avz_mask_features):
    layout "unet"   -> [B, 2, F, T]: log(|Y0| + 1e-7), angle(Y0) - angle(Y1)
                       (full_audio_generating_pipeline/inference.py:90-94);
    layout "tflite" -> [B, F, T, 4]: log_mag, sin(ipd), cos(ipd), linspace(0, 1, F)
                       (Final_pipeline/src/inference.py:198-203, 117-128)."""
    if x.dim() != 3 or x.shape[1] != 2 or x.dtype != torch.float32 or x.stride(2) != 1 \
            or not x.is_cuda:
        raise ValueError("x must be float32 [B, 2, S] on the device")
    B, _, S = x.shape
    if lengths is None:
        lengths = torch.full((B,), S, dtype=torch.int32, device=x.device)
        max_len = S
    if max_len is None:
        max_len = int(lengths.max().item())
    T = n_frames(max_len, plan.hop)
    F = plan.F
    if layout == "unet":
        out = torch.zeros((B, 2, F, T), dtype=torch.float32, device=x.device)
        sb, sc, sf, st = out.stride()
    elif layout == "tflite":
        out = torch.zeros((B, F, T, 4), dtype=torch.float32, device=x.device)
        sb, sf, st, sc = out.stride()
    else:
        raise ValueError(f"unknown feature layout {layout!r}")
    check(lib.avz_mask_features(plan._h, FEATURE_LAYOUTS[layout], B,
                                ct.c_void_p(lengths.data_ptr()), int(max_len),
                                ct.c_void_p(x.data_ptr()), x.stride(0), x.stride(1),
                                ct.c_void_p(out.data_ptr()), sb, sc, sf, st,
                                _stream_handle(stream)), "avz_mask_features")
    return out


def srp_scan(plan: MVDRPlan, mix: torch.Tensor, lengths=None, max_len=None, n_angles=181,
             angle_lo=0.0, angle_hi=180.0, f_lo=200.0, f_hi=4000.0, stream=None):
    """scripts/debug_srp.py:46-62 for a [B, 2, S] batch -> power map [B, n_angles] in dB
    relative to each utterance's maximum (float64, device)."""
    if mix.dim() != 3 or mix.shape[1] != 2 or mix.dtype != torch.float32 or not mix.is_cuda \
            or mix.stride(2) != 1:
        raise ValueError("mix must be float32 [B, 2, S] on the device")
    B, _, S = mix.shape
    if lengths is None:
        lengths = torch.full((B,), S, dtype=torch.int32, device=mix.device)
        max_len = S
    if max_len is None:
        max_len = int(lengths.max().item())
    out = torch.empty((B, n_angles), dtype=torch.float64, device=mix.device)
    check(lib.avz_srp_scan(plan._h, B, ct.c_void_p(lengths.data_ptr()), int(max_len),
                           ct.c_void_p(mix.data_ptr()), mix.stride(0), mix.stride(1), n_angles,
                           float(angle_lo), float(angle_hi), float(f_lo), float(f_hi),
                           ct.c_void_p(out.data_ptr()), _stream_handle(stream)), "avz_srp_scan")
    return out
