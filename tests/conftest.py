import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "real-time-audio-visual-zooming_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def triple_f32(name, seg=None):
    """Bundled reference triple as the reference reads it (int16/32768 -> float32)."""
    g = golden(f"inputs_{name}.npz")
    m, t, i = g["mix"], g["tgt"], g["int"]
    if seg is not None:
        m, t, i = m[seg[0]:seg[1]], t[seg[0]:seg[1]], i[seg[0]:seg[1]]
    f = lambda a: (a.astype(np.float64) / 32768.0).astype(np.float32)  # noqa: E731
    return f(m).T.copy(), f(t), f(i)


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
