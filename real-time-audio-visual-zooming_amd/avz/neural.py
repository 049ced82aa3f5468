"""Neural-mask MVDR path (BASELINE configs[4]) on the MI355X engine: mirror of
rt_av_zoom/core/full_audio_generating_pipeline/inference.py.

Reference, per 2-s chunk (process_chunk, :88-118): STFT 1024/512 -> U-Net input
[log(|Y0| + 1e-7), angle(Y0) - angle(Y1)] -> ``FreqPreservingUNet`` target mask M ->
noise covariance weighted by 1 - M -> MVDR (sigma 1e-5, f < 100 Hz left zero) ->
x max(M, 0.05) -> iSTFT; main_deploy (:120-167) slides 32000-sample windows every 16000
samples (zero-padded tail) and overlap-adds the first 32000 output samples of each,
divided by the per-sample count. No peak normalisation.

Here every chunk of every utterance is one batch item:
  avz_chunk_split -> avz_mask_features (U-Net layout, HIP) -> U-Net forward
  (PyTorch-ROCm, on device, micro-batched) -> avz_mvdr_batch (AVZ_MASK_EXTERNAL,
  AVZ_PF_EXT_FLOOR) -> avz_chunk_merge.
The U-Net is the reference architecture with the reference's module names, so a
state_dict trained upstream (mask_3.pth, absent from the reference checkout) loads
as-is; its forward is PyTorch (MIOpen convolutions), the only part of the path that is
not a hand-written kernel.
"""
from __future__ import annotations

import ctypes as ct
import json
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import wavio
from ._lib import check, lib
from .engine import MVDRPlan, _stream_handle, mask_features
from .final_pipeline import chunk_table

# full_audio_generating_pipeline/config.json (read by inference.py:15-26)
CONF = {"fs": 16000, "n_fft": 1024, "hop_len": 512, "d": 0.04, "c": 343.0,
        "train_seg_samples": 32000}
ANGLE_TARGET = 90.0   # inference.py:24
SIGMA = 1e-5          # inference.py:25
MASK_FLOOR = 0.05     # inference.py:116
FMIN_HZ = 100.0       # inference.py:103


def load_config(path: str = "config.json") -> dict:
    """The reference reads config.json at import (:15-16); here it is optional."""
    if os.path.exists(path):
        with open(path) as fh:
            return {**CONF, **json.load(fh)}
    return dict(CONF)


def _double_conv(cin: int, cout: int) -> nn.Sequential:
    """(3x3 conv, BN, ReLU) x 2 — module layout of FreqPreservingUNet._conv (:45-49)."""
    layers = []
    for a, b in ((cin, cout), (cout, cout)):
        layers += [nn.Conv2d(a, b, 3, padding=1), nn.BatchNorm2d(b), nn.ReLU()]
    return nn.Sequential(*layers)


class FreqPreservingUNet(nn.Module):
    """U-Net over [B, 2, F, T] that pools / upsamples along time only, keeping all F
    bins; sigmoid target mask [B, F, T]. Same submodule names and construction order
    as inference.py:29-67 (state_dict compatible, identical init under one seed)."""

    def __init__(self):
        super().__init__()
        self.pool = nn.MaxPool2d(kernel_size=(1, 2))
        widths = [(2, 32), (32, 64), (64, 128)]
        self.enc1, self.enc2, self.enc3 = (_double_conv(a, b) for a, b in widths)
        self.bot = _double_conv(128, 256)
        for lvl, (c_hi, c_lo) in ((3, (256, 128)), (2, (128, 64)), (1, (64, 32))):
            setattr(self, f"up{lvl}", nn.ConvTranspose2d(c_hi, c_lo, (1, 2), stride=(1, 2)))
            setattr(self, f"dec{lvl}", _double_conv(2 * c_lo, c_lo))
        self.out = nn.Sequential(nn.Conv2d(32, 1, 1), nn.Sigmoid())

    @staticmethod
    def _match(x, skip):
        # nearest resize when pooling dropped an odd frame (:51-54)
        return F.interpolate(x, size=skip.shape[2:], mode="nearest") \
            if x.shape[3] != skip.shape[3] else x

    def forward(self, x):
        skips = []
        for enc in (self.enc1, self.enc2, self.enc3):
            x = enc(x if not skips else self.pool(x))
            skips.append(x)
        x = self.bot(self.pool(x))
        for lvl, skip in zip((3, 2, 1), reversed(skips)):
            up = getattr(self, f"up{lvl}")(x)
            x = getattr(self, f"dec{lvl}")(torch.cat([self._match(up, skip), skip], dim=1))
        return self.out(x).squeeze(1)


def fold_batchnorm(model: nn.Module) -> nn.Module:
    """Inference copy of an eval-mode model with every (Conv2d, BatchNorm2d) pair of its
    Sequential blocks folded into one Conv2d (w * g / sqrt(v + eps), (b - m) g / sqrt(v +
    eps) + beta; torch.nn.utils.fusion.fuse_conv_bn_eval) and the BatchNorm replaced by
    Identity: the U-Net's 14 BatchNorm launches per forward disappear. Module names are
    unchanged; the result differs from the unfolded model by fp32 rounding only."""
    import copy

    from torch.nn.utils.fusion import fuse_conv_bn_eval
    if model.training:
        raise ValueError("fold_batchnorm needs an eval-mode model")
    m = copy.deepcopy(model)
    for seq in m.modules():
        if not isinstance(seq, nn.Sequential):
            continue
        for i in range(len(seq) - 1):
            if isinstance(seq[i], nn.Conv2d) and isinstance(seq[i + 1], nn.BatchNorm2d):
                seq[i] = fuse_conv_bn_eval(seq[i], seq[i + 1])
                seq[i + 1] = nn.Identity()
    return m


class NeuralMaskBeamformer:
    """Batched main_deploy core: [B, 2, S] device mixtures -> [B, S] enhanced signals.

    ``model``: a [n, 2, F, T] -> [n, F, T] mask network on the device (default:
    FreqPreservingUNet in eval mode). ``model_batch`` bounds the chunks per forward.
    ``model_dtype``: torch.float32 (reference precision) or torch.bfloat16 (the forward
    runs in bf16, the mask is handed to the HIP chain in fp32). ``channels_last``: NHWC
    activations for the convolutions (fp32 results equal to within 1e-7 of NCHW on MI355X,
    ~3 % faster forward; tools/unet_speed.py). ``fold_bn``: an eval-mode model runs as its
    BatchNorm-folded copy (fold_batchnorm): the beamformer then holds a SNAPSHOT of the
    weights, so later load_state_dict calls or edits on the caller's model are not seen --
    call ``refresh(model)`` after changing it (or pass fold_bn=False to run the caller's
    module itself)."""

    def __init__(self, model: nn.Module, max_items: int, conf: dict | None = None,
                 model_batch: int = 256, model_dtype=torch.float32, channels_last: bool = True,
                 fold_bn: bool = True):
        conf = conf or CONF
        self.fold_bn = fold_bn
        self.channels_last = channels_last
        self.refresh(model)
        self.chunk = int(conf["train_seg_samples"])
        self.hop_c = self.chunk // 2
        self.model_batch = model_batch
        self.model_dtype = model_dtype
        self.plan = MVDRPlan(n_fft=int(conf["n_fft"]), fs=int(conf["fs"]), mic_d=float(conf["d"]),
                             c_sound=float(conf["c"]), angle_deg=ANGLE_TARGET, sigma=SIGMA,
                             fmin_hz=FMIN_HZ, mask="external", postfilter="floor",
                             pf_floor=MASK_FLOOR, weight_eps=0.0, normalize="none",
                             max_batch=max_items, max_samples=self.chunk)
        # main_deploy keeps the first min(len(out_chunk), WIN_SIZE) samples (:151-153)
        self.item_out_len = min(self.plan.out_len(self.chunk), self.chunk)

    def refresh(self, model: nn.Module) -> None:
        """(Re)build the module the forward runs from ``model``: its BatchNorm-folded copy
        (fold_bn, eval mode), in channels-last memory format if requested."""
        if self.fold_bn and not model.training and any(
                isinstance(x, nn.BatchNorm2d) for x in model.modules()):
            model = fold_batchnorm(model)
        if self.channels_last:
            model = model.to(memory_format=torch.channels_last)
        self.model = model

    @torch.no_grad()
    def masks(self, items: torch.Tensor) -> torch.Tensor:
        """Target masks [n, F, T] (float32) of chunk items [n, 2, chunk]."""
        feats = mask_features(self.plan, items, "unet")
        out = torch.empty((feats.shape[0],) + feats.shape[2:], dtype=torch.float32,
                          device=items.device)
        for s in range(0, feats.shape[0], self.model_batch):
            x = feats[s:s + self.model_batch]
            if self.channels_last:
                x = x.contiguous(memory_format=torch.channels_last)
            if self.model_dtype != torch.float32:
                with torch.autocast("cuda", dtype=self.model_dtype):
                    out[s:s + len(x)] = self.model(x).float()
            else:
                out[s:s + len(x)] = self.model(x)
        return out

    def beamform(self, items: torch.Tensor, mask: torch.Tensor, stream=None) -> torch.Tensor:
        """process_chunk's MVDR + post-filter + iSTFT for every item (one chain launch)."""
        out, _ = self.plan.run(items, ext_mask=mask, stream=stream)
        return out

    def split(self, mix: torch.Tensor, lengths=None, stream=None):
        """main_deploy's sliding windows (:137-147) of a [B, 2, S] batch as chunk items
        [n, 2, chunk] (avz_chunk_split). Returns (items, lengths, d_len, base)."""
        B, _, S = mix.shape
        dev = mix.device
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
                                  _stream_handle(stream)), "avz_chunk_split")
        return items, lengths, d_len, base

    def run(self, mix: torch.Tensor, lengths=None, mask_fn=None, stream=None):
        """mix [B, 2, S] float32 device; lengths: host sequence (default S).
        mask_fn(items) -> [n, F, T] overrides the U-Net. Returns (y [B, S], peak [B])."""
        B, _, S = mix.shape
        dev = mix.device
        st = _stream_handle(stream)
        items, lengths, d_len, base = self.split(mix, lengths, stream)
        mask = mask_fn(items) if mask_fn is not None else self.masks(items)
        item_out = self.beamform(items, mask, stream=stream)
        y = torch.zeros((B, S), dtype=torch.float32, device=dev)
        peak = torch.empty((B,), dtype=torch.float32, device=dev)
        check(lib.avz_chunk_merge(B, max(lengths), self.hop_c, self.item_out_len,
                                  ct.c_void_p(d_len.data_ptr()), ct.c_void_p(base.data_ptr()),
                                  ct.c_void_p(item_out.data_ptr()), item_out.stride(0),
                                  ct.c_void_p(y.data_ptr()), y.stride(0),
                                  ct.c_void_p(peak.data_ptr()), 0, 0.0, st), "avz_chunk_merge")
        return y, peak


def load_model(path: str | None = "mask_3.pth", device=None) -> nn.Module:
    """FreqPreservingUNet in eval mode on the device; weights from ``path`` when given
    (torch.load with weights_only=True: a plain state_dict, as inference.py:131 saves)."""
    model = FreqPreservingUNet()
    if path is not None:
        model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    return model.eval().to(device or torch.device("cuda", torch.cuda.current_device()))


def calculate_metrics_manual(output, target, interf):
    """inference.py:77-85 (the neural script's own SIR: all three signals normalised
    with +1e-6, returns (sir, sir))."""
    if len(target) == 0:
        return 0, 0
    o = output / (np.linalg.norm(output) + 1e-6)
    t = target / (np.linalg.norm(target) + 1e-6)
    i = interf / (np.linalg.norm(interf) + 1e-6)
    p_t = np.sum(np.dot(o, t) ** 2)
    p_i = np.sum(np.dot(o, i) ** 2) + 1e-10
    return 10 * np.log10(p_t / p_i), 10 * np.log10(p_t / p_i)


def main_deploy(input_path: str, model_path: str = "mask_3.pth", model=None,
                conf: dict | None = None):
    """inference.py:120-167 on the engine: reads the stereo mixture, writes
    enhanced_<basename> next to the working directory and returns the output."""
    print(f"Processing {input_path}...")
    if model is None and not os.path.exists(model_path):
        print("Model not found.")
        return None
    conf = conf or load_config()
    y_full, fs = wavio.read(input_path, dtype="float32")
    dev = torch.device("cuda", torch.cuda.current_device())
    model = model if model is not None else load_model(model_path, dev)
    S = y_full.shape[0]
    n_items = -(-S // (int(conf["train_seg_samples"]) // 2))
    print(f"Audio Length: {S / conf['fs']:.2f}s. Processing {n_items} sliding windows...")
    bf = NeuralMaskBeamformer(model, max_items=n_items, conf=conf)
    mix = torch.from_numpy(np.ascontiguousarray(y_full.T))[None].to(dev)
    out, _ = bf.run(mix)
    final = out[0].cpu().numpy()
    out_name = f"enhanced_{os.path.basename(input_path)}"
    wavio.write(out_name, final, fs)
    print(f"Saved: {out_name}")
    if "mixture_" in input_path:
        tgt, _ = wavio.read("target_ref_TEST.wav")
        intf, _ = wavio.read("interf_ref_TEST.wav")
        L = min(len(final), len(tgt))
        sir, _ = calculate_metrics_manual(final[:L], tgt[:L], intf[:L])
        print(f"SIR Improvement: {sir:.2f} dB")
    return final
