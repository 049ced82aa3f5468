"""The reference-side ctypes shim printed in INTEGRATION.md §3, executed as written (only
the library path substituted) against the reference's own outputs: `oracle_mvdr` for the
body of oracle_debug.main (rt_av_zoom/core/oracle_debug.py:42-94) and `batch_mvdr` for
rt_av_zoom/core/tf_lite_version/inference.py:85-179. Tolerances as the parity tests that
go through avz.MVDRPlan: waveform 1e-4 absolute, spectral output 1e-5 of its peak."""
import os
import re
import textwrap

import numpy as np
import pytest

from conftest import ROOT, golden, triple_f32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def shim(gpu_device):
    from avz import _lib
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = textwrap.dedent(re.findall(r"```python\n(.*?)```", text, re.S)[0])
    assert '"/path/to/libavz.so"' in code
    ns = {}
    exec(compile(code.replace('"/path/to/libavz.so"', repr(_lib.LIB_PATH)), "avz_backend", "exec"),
         ns)
    return ns


@pytest.mark.parametrize("name", ["excerpt_test_n512_s1.npz", "excerpt_set2_n1024_s1.npz"])
def test_oracle_mvdr_shim_matches_reference(shim, name):
    g = golden(name)
    mix, tgt, itf = triple_f32(name.split("_")[1], g["seg"])
    out = shim["oracle_mvdr"](mix, tgt, itf, n_fft=int(g["n_fft"]), sigma=float(g["sigma"]))
    ref = g["out"].astype(np.float64)
    assert out.shape == ref.shape
    assert np.max(np.abs(out - ref)) <= 1e-4


@pytest.mark.parametrize("name", ["test_soft", "test_singular"])
def test_batch_mvdr_shim_matches_reference(shim, name):
    g = golden(f"spectral_{name}.npz")
    S = shim["batch_mvdr"](g["Y"], g["mask"], g["f_bins"], g["d_vectors"][:, :, None],
                           float(g["sigma"]))
    ref = g["S_out"].astype(np.complex128)
    assert S.shape == ref.shape and S.dtype == np.complex128
    assert np.abs(S - ref).max() <= 1e-5 * np.abs(ref).max()
