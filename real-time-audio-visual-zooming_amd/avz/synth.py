"""Deterministic synthetic 2-mic scenes (the bench/test input generator).

LJ-Speech cannot be fetched offline, so sources are "speech-like" (SURVEY.md 8(d)):
Gaussian noise -> AR(2) spectral tilt (poles 0.9, 0.5) x a 4 Hz syllabic envelope
with 25 % of 250-ms blocks silenced; rng seed 1000 + utterance index.

Mixing follows the reference's anechoic far-field model:
* delays  — full_audio_generating_pipeline/world_building.py:47-51
* frac delay by rfft phase shift — world_building.py:53-59
* interference gain for SIR 0 dB on mic 1 — Final_pipeline/src/simulation.py:167-179
* AWGN per channel at SNR 5 dB — simulation.py:47-56, world.py:25, 93-98
* shared peak normalisation of mix and refs — simulation.py:197-202
* refs = mic-1 target and mic-1 total interference (world.py:236-238).
Geometry: D = 0.08 m (Final_pipeline/src/config.py:29), target 90 deg,
interferer 1 at 40 deg (world.py:33), further interferers uniform in [0, 180].
"""
from __future__ import annotations

import numpy as np
from scipy.signal import lfilter

FS = 16000
C_SOUND = 343.0
MIC_D = 0.08


def speech_like(rng: np.random.Generator, n: int, fs: int = FS) -> np.ndarray:
    x = rng.standard_normal(n)
    # AR(2) with poles 0.9, 0.5: y[n] = 1.4 y[n-1] - 0.45 y[n-2] + x[n]
    y = lfilter([1.0], [1.0, -1.4, 0.45], x)
    t = np.arange(n) / fs
    env = np.abs(np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, np.pi)))
    blk = int(0.25 * fs)
    nb = -(-n // blk)
    keep = rng.random(nb) >= 0.25
    env *= np.repeat(keep, blk)[:n]
    return y * env


def far_field_delays(azimuth_deg: float, d: float = MIC_D, c: float = C_SOUND):
    th = np.deg2rad(azimuth_deg)
    return (d / 2) * np.cos(th - 0) / c, (d / 2) * np.cos(th - np.pi) / c


def frac_delay(y: np.ndarray, delay_s: float, fs: int = FS) -> np.ndarray:
    n = len(y)
    Yf = np.fft.rfft(y)
    f = np.fft.rfftfreq(n, 1.0 / fs)
    return np.fft.irfft(Yf * np.exp(-1j * 2 * np.pi * f * delay_s), n=n)


def add_awgn(rng: np.random.Generator, s: np.ndarray, snr_db: float) -> np.ndarray:
    p = np.mean(s ** 2)
    if p == 0:
        return s
    return s + rng.normal(0, np.sqrt(p / (10 ** (snr_db / 10))), s.shape)


def make_scene(idx: int, n_samples: int = 64000, n_interferers: int = 1, d: float = MIC_D,
               sir_db: float = 0.0, snr_db: float = 5.0, fs: int = FS):
    """One utterance. Returns (mix [2, S], target_ref [S], interference_ref [S]) float32."""
    rng = np.random.default_rng(1000 + idx)
    angles = [40.0] + list(rng.uniform(0.0, 180.0, max(0, n_interferers - 1)))
    tgt = speech_like(rng, n_samples, fs)
    t1, t2 = far_field_delays(90.0, d)
    tgt_m = [frac_delay(tgt, t1, fs), frac_delay(tgt, t2, fs)]
    int_m = [np.zeros(n_samples), np.zeros(n_samples)]
    for a in angles[:n_interferers]:
        s = speech_like(rng, n_samples, fs)
        d1, d2 = far_field_delays(a, d)
        int_m[0] += frac_delay(s, d1, fs)
        int_m[1] += frac_delay(s, d2, fs)
    p_t, p_i = np.mean(tgt_m[0] ** 2), np.mean(int_m[0] ** 2)
    if n_interferers > 0 and p_i > 0:
        g = np.sqrt(p_t / (p_i * 10 ** (sir_db / 10)))
        int_m = [g * int_m[0], g * int_m[1]]
    mix = np.stack([add_awgn(rng, tgt_m[0] + int_m[0], snr_db),
                    add_awgn(rng, tgt_m[1] + int_m[1], snr_db)])
    peak = np.max(np.abs(mix)) + 1e-9
    return ((mix / peak).astype(np.float32), (tgt_m[0] / peak).astype(np.float32),
            (int_m[0] / peak).astype(np.float32))


def write_world_scene(out_dir: str, mix: np.ndarray, tgt: np.ndarray, itf: np.ndarray,
                      fs: int = FS) -> str:
    """rt_av_zoom/core/world.py:236-263 on-disk format (what oracle_debug.py:35-39 and
    masked_mvdr.py read): stereo ``mixture.wav`` [S, 2] and the mic-1 references as mono
    ``target_reference.wav`` / ``interference_reference.wav``, each reference peak-normalised
    on its own (world.py:243-244). 16-bit PCM like soundfile's WAV default."""
    import os

    from . import wavio
    os.makedirs(out_dir, exist_ok=True)
    wavio.write(os.path.join(out_dir, "mixture.wav"), np.asarray(mix).T, fs)
    for name, r in (("target_reference.wav", tgt), ("interference_reference.wav", itf)):
        r = np.asarray(r, np.float64)
        wavio.write(os.path.join(out_dir, name), r / (np.max(np.abs(r)) + 1e-9), fs)
    return out_dir


def write_final_pipeline_scene(save_dir: str, mix: np.ndarray, tgt: np.ndarray,
                               itf: np.ndarray, tgt2: np.ndarray | None = None,
                               itf2: np.ndarray | None = None, fs: int = FS) -> str:
    """Final_pipeline/src/simulation.py:191-211 format (what run.py inf / eval read):
    stereo ``mixture.wav``, ``target.wav`` and ``interference.wav``, all divided by the
    mixture's peak (the arrays here are already on that shared scale, make_scene).
    ``tgt2``/``itf2`` are the mic-2 images (default: the mic-1 ones). Returns mixture.wav."""
    import os

    from . import wavio
    os.makedirs(save_dir, exist_ok=True)
    tgt2 = tgt if tgt2 is None else tgt2
    itf2 = itf if itf2 is None else itf2
    wavio.write(os.path.join(save_dir, "mixture.wav"), np.asarray(mix).T, fs)
    wavio.write(os.path.join(save_dir, "target.wav"), np.stack([tgt, tgt2], axis=1), fs)
    wavio.write(os.path.join(save_dir, "interference.wav"), np.stack([itf, itf2], axis=1), fs)
    return os.path.join(save_dir, "mixture.wav")


def mix_and_save(sources, prefix: str, angles=(90.0, 40.0, 130.0), d: float = 0.04,
                 fs: int = FS, out_dir: str = "."):
    """full_audio_generating_pipeline/world_building.py:68-100 for given mono sources
    (target first): far-field fractional delays per mic, mic-1 target / interference
    references, shared peak normalisation; writes mixture_<prefix>.wav (stereo),
    target_ref_<prefix>.wav, interf_ref_<prefix>.wav. Returns (mix [2, S], tgt, itf)."""
    import os

    from . import wavio
    n = max(len(s) for s in sources)
    # sources keep their dtype: the reference loads float32 (world_building.py:62), so its
    # forward rfft runs in single precision (numpy >= 2)
    raws = [np.pad(np.asarray(s), (0, n - len(s))) for s in sources]
    m1, m2, tgt_ref, int_ref = (np.zeros(n) for _ in range(4))
    for i, (r, a) in enumerate(zip(raws, angles)):
        t1, t2 = far_field_delays(a, d)
        s1 = frac_delay(r, t1, fs)
        m1 += s1
        m2 += frac_delay(r, t2, fs)
        if i == 0:
            tgt_ref += s1
        else:
            int_ref += s1
    mix = np.stack([m1, m2])
    norm = np.max(np.abs(mix)) + 1e-9
    wavio.write(os.path.join(out_dir, f"mixture_{prefix}.wav"), (mix / norm).T, fs)
    wavio.write(os.path.join(out_dir, f"target_ref_{prefix}.wav"), tgt_ref / norm, fs)
    wavio.write(os.path.join(out_dir, f"interf_ref_{prefix}.wav"), int_ref / norm, fs)
    return mix / norm, tgt_ref / norm, int_ref / norm


def scene_draws(idx: int, n_samples: int = 64000, n_interferers: int = 1, fs: int = FS):
    """The random draws of make_scene(idx) in its RNG order: angles [1 + K] (target 90
    deg first), sources [1 + K, S] and the unit-normal AWGN draws [2, S] (rng.normal(0, s)
    is s * standard_normal in numpy's Generator, so the device scales these)."""
    rng = np.random.default_rng(1000 + idx)
    angles = [40.0] + list(rng.uniform(0.0, 180.0, max(0, n_interferers - 1)))
    srcs = [speech_like(rng, n_samples, fs)]
    for _ in angles[:n_interferers]:
        srcs.append(speech_like(rng, n_samples, fs))
    z = np.stack([rng.standard_normal(n_samples), rng.standard_normal(n_samples)])
    return np.array([90.0] + angles[:n_interferers]), np.stack(srcs), z


def make_batch_device(batch: int, start: int = 0, n_samples: int = 64000,
                      n_interferers: int = 2, d: float = MIC_D, sir_db: float = 0.0,
                      snr_db: float = 5.0, fs: int = FS, device=None):
    """make_batch on the device: the host draws the sources and noise (same RNG stream
    as make_scene), avz_scene_mix does the fractional delays, SIR gain, AWGN and peak
    normalisation. Returns device tensors (mix [B, 2, S], tgt [B, S], itf [B, S])."""
    import ctypes as ct

    import torch

    from ._lib import check, lib
    from .engine import _stream_handle
    dev = device or torch.device("cuda", torch.cuda.current_device())
    K = n_interferers
    angles = np.empty((batch, 1 + K))
    srcs = np.empty((batch, 1 + K, n_samples), np.float32)
    noise = np.empty((batch, 2, n_samples), np.float32)
    for b in range(batch):
        angles[b], srcs[b], noise[b] = scene_draws(start + b, n_samples, K, fs)
    d_ang = torch.from_numpy(angles).to(dev)
    d_src = torch.from_numpy(srcs).to(dev)
    d_noise = torch.from_numpy(noise).to(dev)
    mix = torch.empty((batch, 2, n_samples), dtype=torch.float32, device=dev)
    tgt = torch.empty((batch, n_samples), dtype=torch.float32, device=dev)
    itf = torch.empty((batch, n_samples), dtype=torch.float32, device=dev)
    ws_bytes = lib.avz_scene_workspace_bytes(batch, 1 + K, n_samples)
    ws = torch.empty((max(ws_bytes, 4) + 3) // 4, dtype=torch.float32, device=dev)
    p = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    check(lib.avz_scene_mix(batch, 1 + K, n_samples, p(d_src), p(d_ang), p(d_noise), d, C_SOUND,
                            float(fs), sir_db, snr_db, p(mix), mix.stride(0), mix.stride(1),
                            p(tgt), p(itf), tgt.stride(0), p(ws), ws_bytes,
                            _stream_handle(None)), "avz_scene_mix")
    return mix, tgt, itf


def make_batch(batch: int, start: int = 0, n_samples: int = 64000, n_interferers: int = 2,
               **kw):
    """[B, 2, S] mix, [B, S] target ref, [B, S] interference ref (float32)."""
    mix = np.empty((batch, 2, n_samples), np.float32)
    tgt = np.empty((batch, n_samples), np.float32)
    itf = np.empty((batch, n_samples), np.float32)
    for b in range(batch):
        mix[b], tgt[b], itf[b] = make_scene(start + b, n_samples, n_interferers, **kw)
    return mix, tgt, itf
