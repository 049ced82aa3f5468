"""The oracle's spectral-domain operators pinned to the reference's own outputs
(tests/golden/spectral_*.npz, written by make_golden.py running
rt_av_zoom/core/tf_lite_version/inference.py batch_mvdr; hybrid_test.npz holds the
Final_pipeline hybrid_hard_null_bf I/O of chunk 0)."""
import numpy as np
import pytest

from conftest import golden
from oracle import avz_oracle as O

CASES = ["test_ibm", "test_soft", "set2_soft", "test_singular"]


@pytest.mark.parametrize("name", CASES)
def test_batch_mvdr_oracle_matches_reference(name):
    g = golden(f"spectral_{name}.npz")
    d = O.get_all_steering_vectors(g["f_bins"], float(g["angle"]), float(g["d"]), float(g["c"]))
    assert np.abs(d[:, :, 0] - g["d_vectors"]).max() == 0.0
    S = O.batch_mvdr(g["Y"], g["mask"], g["f_bins"], d, float(g["sigma"]))
    ref = g["S_out"]
    assert np.abs(S - ref).max() <= 1e-6 * np.abs(ref).max() + 1e-7
    # the post-filtered istft of the chunk driver (inference.py:347-352)
    _, x = O.istft(S * np.maximum(g["mask"], 0.05), nperseg=int(g["n_fft"]),
                   noverlap=int(g["n_fft"]) - int(g["hop"]))
    assert np.abs(x - g["chunk_out"]).max() <= 1e-6


def test_batch_mvdr_singular_case_takes_global_fallback():
    g = golden("spectral_test_singular.npz")
    assert bool(g["fallback"])
    d = g["d_vectors"]
    # every bin: w = [1 / (conj(d0) + 1e-10), 0] -> S = Y0 / (d0 + 1e-10)
    S = g["Y"][0] / (d[:, 0:1] + 1e-10)
    assert np.abs(S - g["S_out"]).max() <= 1e-6 * np.abs(S).max()


def test_hybrid_operator_matches_reference_chunk0():
    g = golden("hybrid_test.npz")
    S = O.hybrid_hard_null_bf(g["chunk0_Y"], g["chunk0_mask"], g["chunk0_f"])
    ref = g["chunk0_S"]
    close = np.abs(S - ref).max(axis=1) <= 1e-5 * np.abs(ref).max()
    assert close.mean() >= 0.99
