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
FALLBACKS = {"mic0": _lib.FALLBACK_MIC0, "mean": _lib.FALLBACK_MEAN,
             "batch": _lib.FALLBACK_BATCH}
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
    # AVZ_MASK_IBM: certificate constant of the reference-exact decisions (include/avz.h
    # avz_config.ibm_kappa): 0 = the library default, < 0 = fp32 decisions only
    ibm_kappa: float = 0.0
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
        c.ibm_kappa = cfg.ibm_kappa
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

    def set_timing(self, enable: bool = True, analysis_only: bool = False,
                   period: int = 1) -> None:
        """Time each of the chain's four kernels with HIP events carried by their dispatches
        (analysis_only: the analysis kernel alone) on one run() in `period`."""
        mode = (2 if analysis_only else 1) if enable else 0
        check(lib.avz_plan_set_timing_period(self._h, int(period)), "avz_plan_set_timing_period")
        check(lib.avz_plan_set_timing(self._h, mode), "avz_plan_set_timing")

    def set_ibm_stats(self, counts) -> None:
        """Diagnostics of the exact IBM path: every later run() adds to counts[0] the frames
        and to counts[1] the (bin, frame) decisions taken there (a zeroed int64 CUDA tensor of
        2 elements; None = off)."""
        if counts is not None:
            assert counts.dtype == torch.int64 and counts.is_cuda and counts.numel() >= 2
        check(lib.avz_plan_set_ibm_stats(self._h, _ptr(counts)), "avz_plan_set_ibm_stats")
        self._ibm_stats = counts  # keep the buffer alive

    def set_diagnostics(self, synth_variant: int = 2, ipf_mode: int = 0) -> None:
        """Kernel-path A/B of this plan's later runs (tests / tools; include/avz.h
        avz_plan_set_diagnostics): synth_variant 2 = per-utterance synthesis solving its own
        bins (default), 1 = after the solve kernel, 0 = chunk grid + finalize; ipf_mode 1 / 2
        force the in-kernel piece finalize's rare paths."""
        check(lib.avz_plan_set_diagnostics(self._h, int(synth_variant), int(ipf_mode)),
              "avz_plan_set_diagnostics")

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

    def _batch_args(self, mix, lengths, max_len, ref_tgt, ref_int, ext_mask, out, peak,
                    cov_out, w_out, workspace, need_out=True):
        """Validated avz_batch_args of a time-domain call (shared by run and the stages)."""
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
        a = AvzBatchArgs()
        if need_out:
            if out is None:
                out = self.alloc_out(B, max_len, dev)
            if peak is None:
                peak = torch.empty((B,), dtype=torch.float32, device=dev)
            if out.dtype != torch.float32 or out.dim() != 2 or out.shape[0] < B or \
                    out.shape[1] < self.out_len(max_len) or out.stride(1) != 1:
                raise ValueError("out must be float32 [>= B, >= out_len(max_len)]")
            if peak.dtype != torch.float32 or peak.numel() < B or not peak.is_contiguous():
                raise ValueError("peak must be a contiguous float32 tensor of >= B entries")
            a.out = out.data_ptr()
            a.out_stride = out.stride(0)
            a.peak = peak.data_ptr()
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
        for name, t, last in (("cov_out", cov_out, 5), ("w_out", w_out, 4)):
            if t is not None and (not t.is_cuda or not t.is_contiguous() or t.numel() < B * self.F * last
                                  or t.dtype != (torch.float64 if last == 5 else torch.float32)):
                raise ValueError(f"{name} must be a contiguous device tensor of "
                                 f"[B, F, {last}] {'float64' if last == 5 else 'float32'}")
        a.cov_out = 0 if cov_out is None else cov_out.data_ptr()
        a.w_out = 0 if w_out is None else w_out.data_ptr()
        if workspace is not None:
            if workspace.dtype != torch.uint8 or not workspace.is_cuda:
                raise ValueError("workspace must be a uint8 device tensor")
            a.workspace = workspace.data_ptr()
            a.workspace_bytes = workspace.numel()
        return a, out, peak

    def run(self, mix: torch.Tensor, lengths: torch.Tensor | None = None, *,
            max_len: int | None = None, ref_tgt=None, ref_int=None, ext_mask=None,
            out: torch.Tensor | None = None, peak: torch.Tensor | None = None,
            cov_out=None, w_out=None, workspace: torch.Tensor | None = None, stream=None):
        """mix: [B, 2, S] float32 (device); lengths: [B] int32 (device, default S).
        ref_tgt/ref_int: [B, S] (IBM); ext_mask: [B, F, T] target probability (EXTERNAL).
        workspace: optional uint8 device tensor of >= workspace_bytes(B, max_len) bytes.
        Returns (out [B, >= out_len], peak [B])."""
        a, out, peak = self._batch_args(mix, lengths, max_len, ref_tgt, ref_int, ext_mask, out,
                                        peak, cov_out, w_out, workspace)
        check(lib.avz_mvdr_batch(self._h, ct.byref(a), _stream_handle(stream)), "avz_mvdr_batch")
        return out, peak

    # ------------------------------------------------------------------ stage exports
    def covariance(self, mix, lengths=None, *, max_len=None, ref_tgt=None, ref_int=None,
                   ext_mask=None, cov_out=None, workspace=None, stream=None) -> torch.Tensor:
        """STFT -> mask -> masked covariance sums (avz_mvdr_covariance): [B, F, 5] float64
        (sum m|y0|^2, sum m|y1|^2, Re/Im sum m y0 conj(y1), sum m); oracle_debug.py:42-64."""
        B = mix.shape[0]
        if cov_out is None:
            cov_out = torch.empty((B, self.F, 5), dtype=torch.float64, device=mix.device)
        a, _, _ = self._batch_args(mix, lengths, max_len, ref_tgt, ref_int, ext_mask, None, None,
                                   cov_out, None, workspace, need_out=False)
        check(lib.avz_mvdr_covariance(self._h, ct.byref(a), _stream_handle(stream)),
              "avz_mvdr_covariance")
        return cov_out

    def solve_covariance(self, cov: torch.Tensor, *, steer=None, w=None, fallback=None,
                         stream=None) -> torch.Tensor:
        """Covariance sums [B, F, 5] float64 -> weights [B, F, 4] float32 (Re w0, Im w0,
        Re w1, Im w1) with the plan's beamformer (avz_solve_covariance; oracle_debug.py:66-79).
        steer: optional [F, 2] complex128 device tensor; fallback: optional [B] int32."""
        if cov.dtype != torch.float64 or cov.dim() != 3 or cov.shape[1:] != (self.F, 5) \
                or not cov.is_contiguous() or not cov.is_cuda:
            raise ValueError("cov must be a contiguous float64 [B, F, 5] device tensor")
        B = cov.shape[0]
        if w is None:
            w = torch.empty((B, self.F, 4), dtype=torch.float32, device=cov.device)
        st = self._steer_ptr(steer)
        fb = self._fallback_ptr(fallback, B)
        check(lib.avz_solve_covariance(self._h, B, ct.c_void_p(cov.data_ptr()),
                                       ct.c_void_p(w.data_ptr()), st, fb, _stream_handle(stream)),
              "avz_solve_covariance")
        return w

    def apply_istft(self, mix, w: torch.Tensor, lengths=None, *, max_len=None, gain=None,
                    out=None, peak=None, workspace=None, stream=None):
        """STFT of mix -> S = w^H y (x gain [B, F, T] when given) -> iSTFT/OLA
        (avz_apply_istft; oracle_debug.py:80-94). Returns (out, peak)."""
        if w.dtype != torch.float32 or not w.is_contiguous() or not w.is_cuda \
                or w.numel() < mix.shape[0] * self.F * 4:
            raise ValueError("w must be a contiguous float32 [B, F, 4] device tensor")
        a, out, peak = self._batch_args(mix, lengths, max_len, None, None, gain, out, peak, None,
                                        None, workspace)
        check(lib.avz_apply_istft(self._h, ct.byref(a), ct.c_void_p(w.data_ptr()),
                                  _stream_handle(stream)), "avz_apply_istft")
        return out, peak

    # ------------------------------------------------------------------ spectral domain
    def _steer_ptr(self, steer):
        if steer is None:
            return None
        if steer.dtype != torch.complex128 or steer.shape != (self.F, 2) or not steer.is_cuda \
                or not steer.is_contiguous():
            raise ValueError("steer must be a contiguous complex128 [F, 2] device tensor")
        return ct.c_void_p(steer.data_ptr())

    def _fallback_ptr(self, fallback, B):
        if fallback is None:
            return None
        if fallback.dtype != torch.int32 or fallback.numel() < B or not fallback.is_cuda:
            raise ValueError("fallback must be an int32 device tensor of >= B entries")
        return ct.c_void_p(fallback.data_ptr())

    def beamform_spectral(self, Y: torch.Tensor, mask: torch.Tensor, *, steer=None, S=None,
                          cov_out=None, w_out=None, fallback=None, stream=None) -> torch.Tensor:
        """Y [B, 2, F, T] complex64, mask [B, F, T] float32 target probability -> S [B, F, T]
        complex64 (avz_beamform_spectral: batch_mvdr or hybrid_hard_null_bf per the plan's
        beamformer, the plan's post-filter fused)."""
        if Y.dtype != torch.complex64 or Y.dim() != 4 or Y.shape[1] != 2 or Y.shape[2] != self.F \
                or Y.stride(3) != 1 or not Y.is_cuda:
            raise ValueError(f"Y must be complex64 [B, 2, {self.F}, T] (t contiguous) on the device")
        B, _, _, T = Y.shape
        if mask.dtype != torch.float32 or mask.dim() != 3 or tuple(mask.shape) != (B, self.F, T) \
                or mask.stride(2) != 1 or not mask.is_cuda:
            raise ValueError(f"mask must be float32 [{B}, {self.F}, {T}] (t contiguous)")
        if S is None:
            S = torch.empty((B, self.F, T), dtype=torch.complex64, device=Y.device)
        if S.dtype != torch.complex64 or tuple(S.shape) != (B, self.F, T) or S.stride(2) != 1:
            raise ValueError("S must be complex64 [B, F, T] (t contiguous)")
        for name, t, last, dt in (("cov_out", cov_out, 5, torch.float64),
                                  ("w_out", w_out, 4, torch.float32)):
            if t is not None and (t.dtype != dt or not t.is_contiguous() or not t.is_cuda
                                  or t.numel() < B * self.F * last):
                raise ValueError(f"{name} must be a contiguous [B, F, {last}] {dt} device tensor")
        a = _lib.AvzSpectralArgs()
        a.batch, a.frames = B, T
        a.Y = Y.data_ptr()
        a.y_stride_b, a.y_stride_m, a.y_stride_f = Y.stride(0), Y.stride(1), Y.stride(2)
        a.mask = mask.data_ptr()
        a.mask_stride_b, a.mask_stride_f = mask.stride(0), mask.stride(1)
        st = self._steer_ptr(steer)
        a.steer = st.value if st is not None else None
        a.S = S.data_ptr()
        a.s_stride_b, a.s_stride_f = S.stride(0), S.stride(1)
        a.cov_out = None if cov_out is None else cov_out.data_ptr()
        a.w_out = None if w_out is None else w_out.data_ptr()
        fb = self._fallback_ptr(fallback, B)
        a.fallback = fb.value if fb is not None else None
        check(lib.avz_beamform_spectral(self._h, ct.byref(a), _stream_handle(stream)),
              "avz_beamform_spectral")
        return S

    def istft(self, S: torch.Tensor, *, out=None, peak=None, workspace=None, stream=None):
        """scipy.signal.istft(S, nperseg=n_fft, noverlap=n_fft/2) of S [B, F, T] complex64
        (t contiguous): (out [B, >= (T-1) hop], peak [B]); the plan's normalisation applies."""
        if S.dtype != torch.complex64 or S.dim() != 3 or S.shape[1] != self.F or S.stride(2) != 1 \
                or not S.is_cuda:
            raise ValueError(f"S must be complex64 [B, {self.F}, T] (t contiguous) on the device")
        B, _, T = S.shape
        n = (T - 1) * self.hop
        if out is None:
            out = torch.empty((B, (n + 3) // 4 * 4), dtype=torch.float32, device=S.device)
        if peak is None:
            peak = torch.empty((B,), dtype=torch.float32, device=S.device)
        if out.dtype != torch.float32 or out.dim() != 2 or out.shape[0] < B or out.shape[1] < n \
                or out.stride(1) != 1:
            raise ValueError("out must be float32 [>= B, >= (T - 1) hop]")
        wp, wn = (None, 0) if workspace is None else (ct.c_void_p(workspace.data_ptr()),
                                                       workspace.numel())
        check(lib.avz_istft(self._h, B, T, ct.c_void_p(S.data_ptr()), S.stride(0), S.stride(1),
                            ct.c_void_p(out.data_ptr()), out.stride(0),
                            ct.c_void_p(peak.data_ptr()), wp, wn, _stream_handle(stream)),
              "avz_istft")
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
