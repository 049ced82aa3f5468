"""PCM WAV I/O with the reference's conventions.

* read:  int16 PCM -> float32 / 32768 (libsndfile's mapping, as `sf.read(..., dtype=
  'float32')` in oracle_debug.py:35-39); stereo returns [S, 2] like soundfile.
* write: float -> PCM_16 (soundfile's default WAV subtype used by `sf.write`,
  oracle_debug.py:96): clip to [-1, 1), scale by 32768, round to nearest.
Uses only the standard library `wave` module (libsndfile is not installed).
"""
from __future__ import annotations

import wave

import numpy as np


def read(path: str, dtype="float32"):
    """Returns (data, fs); data [S] (mono) or [S, C] like soundfile.read."""
    with wave.open(path, "rb") as w:
        ch, width, fs, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if width != 2:
        raise ValueError(f"{path}: only 16-bit PCM is supported (got {8 * width}-bit)")
    x = np.frombuffer(raw, dtype="<i2").reshape(-1, ch)
    x = (x.astype(np.float64) / 32768.0).astype(dtype)
    return (x[:, 0] if ch == 1 else x), fs


def write(path: str, data, fs: int) -> None:
    """float [S] or [S, C] -> 16-bit PCM WAV."""
    x = np.asarray(data, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    q = np.clip(np.round(x * 32768.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(q.shape[1])
        w.setsampwidth(2)
        w.setframerate(int(fs))
        w.writeframes(q.tobytes())
