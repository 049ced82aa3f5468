"""Mirror of rt_av_zoom/core/tf_lite_version/inference.py's chunked driver
(process_audio_file, :245-391) on the MI355X engine.

The reference cuts a stereo file into 2-s chunks (WIN_SIZE = 32000 samples every 16000,
ceil(S / 16000) chunks, zero-padded tail), computes per chunk the features
[log(|Y0| + 1e-7), angle(Y0) - angle(Y1)] (:296-298) for a TFLite mask model
(TFLiteBeamformer, :185-239), beamforms with the vectorised ``batch_mvdr`` (:85-179;
sqrt(1 - M + 1e-10) covariance weights, no low-frequency skip, one solve whose
LinAlgError sends the whole chunk to w~ = [1, 0]), multiplies by max(M, 0.05), inverts the
chunk and overlap-adds its WHOLE istft output (32256 samples) at the chunk start with a
per-sample count, then divides by the count and peak-normalises with + 1e-9.

Here every chunk is one item of one chain launch: ``avz_chunk_split`` -> device features
(``avz_mask_features``, NHWC [n, F, T, 2] as the TFLite input) -> the caller's mask model
-> ``avz_mvdr_batch`` (external mask, batch_mvdr semantics, max(M, 0.05) post-filter) ->
``avz_chunk_merge`` (overlap-add / count, peak + 1e-9). The TFLite model itself cannot run
here (TensorFlow absent, model file missing upstream): the mask comes from ``mask_fn``,
any device model taking the features.
"""
from __future__ import annotations

import ctypes as ct
import os
import time

import numpy as np
import torch

from . import wavio
from ._lib import check, lib
from .engine import MVDRPlan, _stream_handle, mask_features
from .final_pipeline import chunk_table

# tf_lite_version/config.json (read by inference.py:9-25) and inference.py:44-48
FS = 16000
N_FFT = 1024
HOP = 512
D = 0.04
C = 343.0
WIN_SIZE = 32000
ANGLE_TARGET = 90.0
SIGMA = 1e-5
N_MICS = 2
MASK_FLOOR = 0.05  # :341


def get_all_steering_vectors(f_bins, angle_deg, d, c):
    """inference.py:53-81: [F, 2, 1] complex128 far-field vectors (host helper; the plan
    evaluates the same expression per bin for the kernels)."""
    th = np.deg2rad(angle_deg)
    om = 2 * np.pi * np.asarray(f_bins)
    sv = np.stack([np.exp(-1j * om * ((d / 2) * np.cos(th) / c)),
                   np.exp(-1j * om * ((d / 2) * np.cos(th - np.pi) / c))], axis=0)
    return np.expand_dims(sv.T, axis=-1)


class ChunkedMVDRBeamformer:
    """Batched process_audio_file core: [B, 2, S] device mixtures -> [B, S] enhanced."""

    def __init__(self, max_items: int, chunk: int = WIN_SIZE, n_fft: int = N_FFT,
                 d: float = D, c: float = C, sigma: float = SIGMA):
        self.chunk = chunk
        self.hop_c = chunk // 2
        self.plan = MVDRPlan(n_fft=n_fft, fs=FS, mic_d=d, c_sound=c, angle_deg=ANGLE_TARGET,
                             sigma=sigma, mask="external", postfilter="floor",
                             pf_floor=MASK_FLOOR, weight_eps=1e-10, fmin_hz=0.0,
                             singular_fallback="batch", normalize="none",
                             max_batch=max_items, max_samples=chunk)
        # the whole istft output of a chunk is overlap-added (inference.py:347-355)
        self.item_out_len = self.plan.out_len(chunk)

    def features(self, items: torch.Tensor, stream=None) -> torch.Tensor:
        """TFLite input tensors [n, F, T, 2] (log_mag, ipd) of chunk items [n, 2, chunk]
        (inference.py:296-298, 201-203)."""
        f = mask_features(self.plan, items, "unet", stream=stream)
        return f.permute(0, 2, 3, 1).contiguous()

    def run(self, mix: torch.Tensor, mask_fn, lengths=None, stream=None):
        """mix [B, 2, S] float32 device; ``mask_fn(features [n, F, T, 2]) -> M [n, F, T]``
        target probability per chunk item (utterance-major, chunk order). Returns
        (y [B, S] float32 peak-normalised with + 1e-9, peak [B] before normalisation)."""
        B, _, S = mix.shape
        dev = mix.device
        st = _stream_handle(stream)
        lengths = [S] * B if lengths is None else [int(x) for x in lengths]
        utt_h, start_h, base_h = chunk_table(lengths, self.hop_c)
        n = len(utt_h)
        utt = torch.from_numpy(utt_h).to(dev)
        start = torch.from_numpy(start_h).to(dev)
        base = torch.from_numpy(base_h).to(dev)
        d_len = torch.tensor(lengths, dtype=torch.int32, device=dev)
        items = torch.empty((n, 2, self.chunk), dtype=torch.float32, device=dev)
        check(lib.avz_chunk_split(n, 2, self.chunk, ct.c_void_p(utt.data_ptr()),
                                  ct.c_void_p(start.data_ptr()), ct.c_void_p(d_len.data_ptr()),
                                  ct.c_void_p(mix.data_ptr()), mix.stride(0), mix.stride(1),
                                  ct.c_void_p(items.data_ptr()), items.stride(0), items.stride(1),
                                  st), "avz_chunk_split")
        mask = mask_fn(self.features(items, stream))
        item_out, _ = self.plan.run(items, ext_mask=mask, stream=stream)
        y = torch.zeros((B, S), dtype=torch.float32, device=dev)
        peak = torch.empty((B,), dtype=torch.float32, device=dev)
        check(lib.avz_chunk_merge(B, max(lengths), self.hop_c, self.item_out_len,
                                  ct.c_void_p(d_len.data_ptr()), ct.c_void_p(base.data_ptr()),
                                  ct.c_void_p(item_out.data_ptr()), item_out.stride(0),
                                  ct.c_void_p(y.data_ptr()), y.stride(0),
                                  ct.c_void_p(peak.data_ptr()), 1, 1e-9, st), "avz_chunk_merge")
        return y, peak


def process_audio_file(input_path, output_path, model_path="mask_estimator.tflite",
                       mask_fn=None):
    """inference.py:245-391 on the engine: reads the stereo WAV, enhances it in one batch
    of chunk items and writes ``output_path`` as 16-bit PCM (libsndfile's default WAV
    subtype, which the reference's sf.write uses). Prints the reference's statistics.

    ``mask_fn(features [n, F, T, 2]) -> M [n, F, T]`` stands in for the TFLite model at
    ``model_path``, which cannot run here (no TensorFlow; the model file is absent
    upstream). As in the reference, a missing ``model_path`` raises FileNotFoundError
    (its size is printed first, :249-251); without ``mask_fn`` the call fails there too."""
    size_mb = os.path.getsize(model_path) / 1024 / 1024
    print(f"Model Size:       {size_mb:.2f} MB")
    if mask_fn is None:
        raise RuntimeError(f"no TFLite runtime for {model_path}: pass mask_fn (a device mask "
                           "model over the [n, F, T, 2] features)")
    y, sr = wavio.read(input_path, dtype="float32")
    if sr != FS:
        print("Warning: SR mismatch")
    print(f"Audio Duration:   {len(y) / FS:.2f}s")
    dev = torch.device("cuda", torch.cuda.current_device())
    S = y.shape[0]
    bf = ChunkedMVDRBeamformer(max_items=-(-S // (WIN_SIZE // 2)))
    mix = torch.from_numpy(np.ascontiguousarray(y.T))[None].to(dev)
    start_time = time.time()
    out, _ = bf.run(mix, mask_fn)
    final = out[0].cpu().numpy()
    proc_time = time.time() - start_time
    wavio.write(output_path, final, FS)
    print("-" * 40)
    print(f"Total Inference Time: {proc_time:.4f}s")
    print(f"Real-Time Factor:     {proc_time / (len(y) / FS):.4f}x")
    print(f"Saved to:             {output_path}")
    print("-" * 40)
    return final
