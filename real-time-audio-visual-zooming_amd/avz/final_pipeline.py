"""Mirror of Final_pipeline/src/inference.py (the beamformer `run.py inf` and
`batch_run.py` call) on the MI355X engine.

The reference's driver (inference.py:144-237) cuts a stereo mixture into 2-s chunks
(WIN_SIZE = 32000 samples every 16000, zero-padded tail), asks a TFLite model for a
target-probability mask per chunk, runs ``hybrid_hard_null_bf`` (inference.py:28-98),
multiplies by the mask, inverts each chunk and overlap-adds the chunk outputs divided
by the per-sample count, then peak-normalises with +1e-9.

Here every chunk of every utterance is one batch item of the HIP chain
(``avz_chunk_split`` -> ``avz_mvdr_batch`` with AVZ_BF_HYBRID_NULL -> ``avz_chunk_merge``):
a batch of B utterances is one chunk split, one beamforming chain launch and one merge.

Mask sources: the TFLite model file is absent from the reference
(.MISSING_LARGE_BLOBS:1) and TensorFlow is not installed, so the mask comes either from
the oracle references (``mask="ibm"``: target mask |S_t| >= |S_i|, exactly the engine's
IBM mode with the x(1 - noise) post-filter) or from any caller-supplied model
(``mask="external"``: ``mask_fn(items [n, 2, chunk]) -> M [n, F, T]``).
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np
import torch

from . import wavio
from ._lib import check, lib
from .engine import MVDRPlan, _stream_handle

# Final_pipeline/src/config.py:14-29 and inference.py:10-12
FS = 16000
C_SPEED = 343.0
N_FFT = 1024
HOP_LEN = 512
WIN_SIZE = 32000
MIC_DIST = 0.08
ANGLE_TARGET = 90.0
FREQ_BINS = N_FFT // 2 + 1
N_MICS = 2
BYPASS_HZ = 200.0   # inference.py:50
COND_MAX = 10.0     # inference.py:80
RESULTS_DIR = os.path.join("data", "results")


def get_steering_vector_single(f, angle_deg, d, c):
    """inference.py:16-26 — (2, 1) complex128, phase-normalised to mic 0 (host helper;
    the plan evaluates the same expression once per bin for the kernels)."""
    th = np.deg2rad(angle_deg)
    om = 2 * np.pi * f
    v = np.array([[np.exp(-1j * om * ((d / 2) * np.cos(th) / c))],
                  [np.exp(-1j * om * ((d / 2) * np.cos(th - np.pi) / c))]])
    return v / (v[0] + 1e-10)


def chunk_table(lengths, hop=WIN_SIZE // 2):
    """Item tables of the driver's chunk loop (inference.py:177-181) for a batch:
    chunks c = 0 .. ceil(L/hop) - 1 of utterance b start at c * hop."""
    utt, start, base = [], [], []
    for b, L in enumerate(int(x) for x in lengths):
        base.append(len(utt))
        n = -(-L // hop)
        utt += [b] * n
        start += [c * hop for c in range(n)]
    return (np.asarray(utt, np.int32), np.asarray(start, np.int32), np.asarray(base, np.int32))


class ChunkedHybridBeamformer:
    """Batched enhance_audio core: [B, 2, S] device mixtures -> [B, S] enhanced."""

    def __init__(self, max_items: int, mask: str = "ibm", chunk: int = WIN_SIZE,
                 n_fft: int = N_FFT, mic_d: float = MIC_DIST, normalize: bool = True,
                 norm_eps: float = 1e-9):
        if mask not in ("ibm", "external"):
            raise ValueError("mask must be 'ibm' (oracle references) or 'external'")
        self.mask = mask
        self.chunk = chunk
        self.hop_c = chunk // 2
        self.normalize = normalize
        self.norm_eps = norm_eps
        self.plan = MVDRPlan(n_fft=n_fft, fs=FS, mic_d=mic_d, c_sound=C_SPEED,
                             angle_deg=ANGLE_TARGET, mask=mask,
                             postfilter="ibm" if mask == "ibm" else "mul",
                             beamformer="hybrid_null", bypass_hz=BYPASS_HZ, cond_max=COND_MAX,
                             normalize="none", weight_eps=0.0, max_batch=max_items,
                             max_samples=chunk)
        self.item_out_len = self.plan.out_len(chunk)

    def _split(self, x, utt, start, lengths, items, channels, stream):
        check(lib.avz_chunk_split(len(utt), channels, self.chunk, ct.c_void_p(utt.data_ptr()),
                                  ct.c_void_p(start.data_ptr()), ct.c_void_p(lengths.data_ptr()),
                                  ct.c_void_p(x.data_ptr()), x.stride(0),
                                  x.stride(1) if channels > 1 else 0,
                                  ct.c_void_p(items.data_ptr()), items.stride(0),
                                  items.stride(1) if channels > 1 else 0, stream),
              "avz_chunk_split")

    def run(self, mix: torch.Tensor, lengths=None, ref_tgt=None, ref_int=None, mask_fn=None,
            stream=None):
        """mix [B, 2, S] float32 device; lengths: host sequence (default S).
        mask="ibm": ref_tgt/ref_int [B, S] (mic-1 references).
        mask="external": mask_fn(items [n, 2, chunk]) -> target probability [n, F, T].
        Returns (y [B, S] float32, peak [B])."""
        B, _, S = mix.shape
        dev = mix.device
        lengths = [S] * B if lengths is None else [int(x) for x in lengths]
        utt_h, start_h, base_h = chunk_table(lengths, self.hop_c)
        n = len(utt_h)
        st = _stream_handle(stream)
        utt = torch.from_numpy(utt_h).to(dev)
        start = torch.from_numpy(start_h).to(dev)
        base = torch.from_numpy(base_h).to(dev)
        d_len = torch.tensor(lengths, dtype=torch.int32, device=dev)
        items = torch.empty((n, 2, self.chunk), dtype=torch.float32, device=dev)
        self._split(mix, utt, start, d_len, items, 2, st)
        kw = {}
        if self.mask == "ibm":
            if ref_tgt is None or ref_int is None:
                raise ValueError("mask='ibm' needs ref_tgt and ref_int")
            it = torch.empty((n, self.chunk), dtype=torch.float32, device=dev)
            ii = torch.empty((n, self.chunk), dtype=torch.float32, device=dev)
            self._split(ref_tgt, utt, start, d_len, it, 1, st)
            self._split(ref_int, utt, start, d_len, ii, 1, st)
            kw = dict(ref_tgt=it, ref_int=ii)
        else:
            if mask_fn is None:
                raise ValueError("mask='external' needs mask_fn")
            kw = dict(ext_mask=mask_fn(items))
        item_out, _ = self.plan.run(items, **kw, stream=stream)
        y = torch.zeros((B, S), dtype=torch.float32, device=dev)
        peak = torch.empty((B,), dtype=torch.float32, device=dev)
        check(lib.avz_chunk_merge(B, max(lengths), self.hop_c, self.item_out_len,
                                  ct.c_void_p(d_len.data_ptr()), ct.c_void_p(base.data_ptr()),
                                  ct.c_void_p(item_out.data_ptr()), item_out.stride(0),
                                  ct.c_void_p(y.data_ptr()), y.stride(0),
                                  ct.c_void_p(peak.data_ptr()), int(self.normalize),
                                  float(self.norm_eps), st), "avz_chunk_merge")
        return y, peak


def enhance_audio(run_name, input_path, model_path=None, mask_fn=None, refs=None,
                  results_dir=RESULTS_DIR):
    """inference.py:144-237 on the engine. Writes
    <results_dir>/<run_name>_results/<run_name>_enhanced.wav as 16-bit PCM (libsndfile's
    default WAV subtype, which the reference's sf.write uses).

    Mask: ``mask_fn`` (a device mask model, see ChunkedHybridBeamformer), else the oracle
    target mask from ``refs`` = (target, interference) mono arrays, else the
    ``target.wav`` / ``interference.wav`` written next to the mixture by
    Final_pipeline/src/simulation.py:205-211 (channel 0 = mic 1). The TFLite model at
    ``model_path`` cannot run here (no TensorFlow, model file absent upstream)."""
    result_dir = os.path.join(results_dir, f"{run_name}_results")
    os.makedirs(result_dir, exist_ok=True)
    output_path = os.path.join(result_dir, f"{run_name}_enhanced.wav")
    print(f"[INF] Processing {input_path}")
    print(f"[INF] Saving to  {output_path}")
    y, sr = wavio.read(input_path, dtype="float32")
    if sr != FS:
        print(f"Warning: SR mismatch. Input: {sr}, Config: {FS}")
    if y.ndim == 1:
        print("Error: Input is mono. Requires 2 channels.")
        return None
    if mask_fn is None and refs is None:
        d = os.path.dirname(input_path)
        tp, ip = os.path.join(d, "target.wav"), os.path.join(d, "interference.wav")
        if not (os.path.exists(tp) and os.path.exists(ip)):
            print(f"Failed to load TFLite model: {model_path} (no TFLite runtime); "
                  "no oracle references next to the mixture either")
            return None
        t, _ = wavio.read(tp, dtype="float32")
        i, _ = wavio.read(ip, dtype="float32")
        refs = (t if t.ndim == 1 else t[:, 0], i if i.ndim == 1 else i[:, 0])
    dev = torch.device("cuda", torch.cuda.current_device())
    S = y.shape[0]
    n_items = -(-S // (WIN_SIZE // 2))
    bf = ChunkedHybridBeamformer(max_items=n_items, mask="external" if mask_fn else "ibm")
    mix = torch.from_numpy(np.ascontiguousarray(y.T))[None].to(dev)
    if mask_fn is not None:
        out, _ = bf.run(mix, mask_fn=mask_fn)
    else:
        def ref(a):
            a = np.asarray(a, np.float32)[:S]
            return torch.from_numpy(np.pad(a, (0, S - len(a))))[None].to(dev)
        out, _ = bf.run(mix, ref_tgt=ref(refs[0]), ref_int=ref(refs[1]))
    final = out[0].cpu().numpy()
    wavio.write(output_path, final, FS)
    print("[INF] Saved successfully.")
    return final
