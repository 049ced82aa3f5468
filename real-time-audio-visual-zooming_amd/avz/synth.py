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


# ---------------------------------------------------------------- counter-based draws
# The device generator (avz_scene_generate, csrc/avz_scene.hip) draws from Philox4x32-10
# streams keyed by (utterance index, SCENE_KEY ^ seed); this is its host restatement.
SCENE_KEY = 0x5CE7E5ED
STREAM_NOISE, STREAM_UNIF = 0x100, 0x200
UNIF_PHASE, UNIF_KEEP = 0x1000, 0x100000
_M32 = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0: int, k1: int):
    """Random123 philox4x32-10 on uint32 counter arrays; returns four uint64 arrays < 2^32."""
    c0, c1, c2, c3 = (np.asarray(c, np.uint64) & _M32 for c in (c0, c1, c2, c3))
    k0, k1 = np.uint64(k0 & 0xFFFFFFFF), np.uint64(k1 & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & _M32, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & _M32
        k0 = (k0 + np.uint64(0x9E3779B9)) & _M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & _M32
    return c0, c1, c2, c3


def _u53(hi, lo):
    return (((hi << np.uint64(32)) | lo) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def _key(idx: int, seed: int = 0):
    return idx & 0xFFFFFFFF, ((idx >> 32) ^ SCENE_KEY ^ seed) & 0xFFFFFFFF


def philox_normals(key, stream: int, n: int) -> np.ndarray:
    """n standard normals of a stream: pair i = Box-Muller of block i's two 53-bit uniforms."""
    i = np.arange((n + 1) // 2, dtype=np.uint64)
    x, y, z, w = philox4x32(i, stream, 0, 0, *key)
    u1 = (((x << np.uint64(32)) | y) >> np.uint64(11)).astype(np.float64)
    u1 = (u1 + 1.0) * 2.0 ** -53
    u2 = _u53(z, w)
    r = np.sqrt(-2.0 * np.log(u1))
    out = np.empty(2 * len(i))
    out[0::2] = r * np.cos(2.0 * np.pi * u2)
    out[1::2] = r * np.sin(2.0 * np.pi * u2)
    return out[:n]


def philox_uniform(key, j) -> np.ndarray:
    x, y, _, _ = philox4x32(np.asarray(j, np.uint64), STREAM_UNIF, 0, 0, *key)
    return _u53(x, y)


def speech_like_philox(key, s: int, n: int, fs: int = FS) -> np.ndarray:
    """speech_like() on the counter-based streams of source s."""
    y = lfilter([1.0], [1.0, -1.4, 0.45], philox_normals(key, s, n))
    phi = np.pi * philox_uniform(key, UNIF_PHASE + s)
    t = np.arange(n) / fs
    env = np.abs(np.sin(2 * np.pi * 4.0 * t + phi))
    blk = int(0.25 * fs)
    nb = -(-n // blk)
    keep = philox_uniform(key, UNIF_KEEP * (1 + s) + np.arange(nb)) >= 0.25
    env *= np.repeat(keep, blk)[:n]
    return y * env


def scene_draws_philox(idx: int, n_samples: int = 64000, n_interferers: int = 1,
                       fs: int = FS, seed: int = 0):
    """(angles [1 + K], sources [1 + K, S], unit-normal noise [2, S]) of utterance idx."""
    key = _key(idx, seed)
    K = n_interferers
    angles = [90.0] + ([40.0] if K >= 1 else [])
    if K > 1:
        angles += list(180.0 * philox_uniform(key, np.arange(K - 1)))
    srcs = np.stack([speech_like_philox(key, s, n_samples, fs) for s in range(1 + K)])
    z = np.stack([philox_normals(key, STREAM_NOISE + c, n_samples) for c in range(2)])
    return np.array(angles), srcs, z


def mix_draws(angles, srcs, z, d: float = MIC_D, sir_db: float = 0.0, snr_db: float = 5.0,
              fs: int = FS):
    """make_scene's mixing (delays, SIR gain on mic 1, AWGN, shared peak) of given draws."""
    n = srcs.shape[-1]
    K = len(angles) - 1
    t1, t2 = far_field_delays(angles[0], d)
    tgt_m = [frac_delay(srcs[0], t1, fs), frac_delay(srcs[0], t2, fs)]
    int_m = [np.zeros(n), np.zeros(n)]
    for k in range(1, K + 1):
        d1, d2 = far_field_delays(angles[k], d)
        int_m[0] += frac_delay(srcs[k], d1, fs)
        int_m[1] += frac_delay(srcs[k], d2, fs)
    p_t, p_i = np.mean(tgt_m[0] ** 2), np.mean(int_m[0] ** 2)
    if K > 0 and p_i > 0:
        g = np.sqrt(p_t / (p_i * 10 ** (sir_db / 10)))
        int_m = [g * int_m[0], g * int_m[1]]
    mix = []
    for c in range(2):
        cl = tgt_m[c] + int_m[c]
        p = np.mean(cl ** 2)
        mix.append(cl if p == 0 else cl + np.sqrt(p / (10 ** (snr_db / 10))) * z[c])
    mix = np.stack(mix)
    peak = np.max(np.abs(mix)) + 1e-9
    return ((mix / peak).astype(np.float32), (tgt_m[0] / peak).astype(np.float32),
            (int_m[0] / peak).astype(np.float32))


def make_scene_philox(idx: int, n_samples: int = 64000, n_interferers: int = 1,
                      d: float = MIC_D, sir_db: float = 0.0, snr_db: float = 5.0,
                      fs: int = FS, seed: int = 0):
    """Host restatement of avz_scene_generate for one utterance (make_scene's model on the
    counter-based draws)."""
    a, s, z = scene_draws_philox(idx, n_samples, n_interferers, fs, seed)
    return mix_draws(a, s, z, d, sir_db, snr_db, fs)


def make_batch_philox(batch: int, start: int = 0, n_samples: int = 64000,
                      n_interferers: int = 2, seed: int = 0, **kw):
    mix = np.empty((batch, 2, n_samples), np.float32)
    tgt = np.empty((batch, n_samples), np.float32)
    itf = np.empty((batch, n_samples), np.float32)
    for b in range(batch):
        mix[b], tgt[b], itf[b] = make_scene_philox(start + b, n_samples, n_interferers,
                                                   seed=seed, **kw)
    return mix, tgt, itf


def make_batch_device(batch: int, start: int = 0, n_samples: int = 64000,
                      n_interferers: int = 2, d: float = MIC_D, sir_db: float = 0.0,
                      snr_db: float = 5.0, fs: int = FS, device=None, rng: str = "host",
                      seed: int = 0):
    """A batch of scenes as device tensors (mix [B, 2, S], tgt [B, S], itf [B, S]).

    rng="host":   make_batch's scenes — the host draws the sources and noise (same RNG
                  stream as make_scene) and avz_scene_mix does the delays, SIR gain, AWGN
                  and peak normalisation.
    rng="philox": avz_scene_generate — draws and all on the device (make_batch_philox is
                  the host restatement); no host work, so a large shard costs milliseconds.
    """
    import ctypes as ct

    import torch

    from ._lib import check, lib
    from .engine import _stream_handle
    dev = device or torch.device("cuda", torch.cuda.current_device())
    K = n_interferers
    mix = torch.empty((batch, 2, n_samples), dtype=torch.float32, device=dev)
    tgt = torch.empty((batch, n_samples), dtype=torch.float32, device=dev)
    itf = torch.empty((batch, n_samples), dtype=torch.float32, device=dev)
    p = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    if rng == "philox":
        ws_bytes = lib.avz_scene_generate_workspace_bytes(batch, K, n_samples)
        ws = torch.empty((max(ws_bytes, 4) + 3) // 4, dtype=torch.float32, device=dev)
        check(lib.avz_scene_generate(batch, start, K, n_samples, seed, d, C_SOUND, float(fs),
                                     sir_db, snr_db, p(mix), mix.stride(0), mix.stride(1), p(tgt),
                                     p(itf), tgt.stride(0), p(ws), ws_bytes,
                                     _stream_handle(None)), "avz_scene_generate")
        return mix, tgt, itf
    if rng != "host":
        raise ValueError(f"rng must be 'host' or 'philox', not {rng!r}")
    angles = np.empty((batch, 1 + K))
    srcs = np.empty((batch, 1 + K, n_samples), np.float32)
    noise = np.empty((batch, 2, n_samples), np.float32)
    for b in range(batch):
        angles[b], srcs[b], noise[b] = scene_draws(start + b, n_samples, K, fs)
    d_ang = torch.from_numpy(angles).to(dev)
    d_src = torch.from_numpy(srcs).to(dev)
    d_noise = torch.from_numpy(noise).to(dev)
    ws_bytes = lib.avz_scene_workspace_bytes(batch, 1 + K, n_samples)
    ws = torch.empty((max(ws_bytes, 4) + 3) // 4, dtype=torch.float32, device=dev)
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
