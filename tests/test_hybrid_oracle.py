"""CPU: the Final_pipeline restatement (oracle/avz_oracle.py hybrid_* / enhance_chunked)
against fixtures produced by running the reference's own enhance_audio
(Final_pipeline/src/inference.py:144-237) with the oracle target mask standing in for the
absent TFLite model (tests/golden/make_golden.py, gen_final_pipeline)."""
import numpy as np
import pytest

from conftest import golden, triple_f32
from oracle import avz_oracle as O


@pytest.fixture(scope="module")
def g_test():
    return golden("hybrid_test.npz")


def test_hybrid_loop_matches_reference_chunk(g_test):
    Y, M, f, S = g_test["chunk0_Y"], g_test["chunk0_mask"], g_test["chunk0_f"], g_test["chunk0_S"]
    W = O.hybrid_weights_loop(Y, M, f)
    S_o = np.einsum("fm,mft->ft", W.conj(), Y)
    assert np.abs(S_o - S).max() <= 1e-6 * np.abs(S).max()


def test_hybrid_closed_form_matches_loop(g_test):
    """The kernels' closed-form algebra (fp64) vs the LAPACK loop (complex64 covariance)."""
    Y, M, f = g_test["chunk0_Y"], g_test["chunk0_mask"], g_test["chunk0_f"]
    Wl = O.hybrid_weights_loop(Y, M, f)
    Wv = O.hybrid_weights_vec(Y, M, f)
    assert np.abs(Wl - Wv).max() < 1e-4
    # same branch (bypass / delay-and-sum / null) on every bin
    ds = lambda W: np.isclose(np.abs(W[:, 0]), 0.5, atol=1e-9)  # noqa: E731
    assert (ds(Wl) == ds(Wv)).all()
    assert (Wl[f < 200] == [1, 0]).all()


def test_hybrid_branch_counts(g_test):
    Y, M, f = g_test["chunk0_Y"], g_test["chunk0_mask"], g_test["chunk0_f"]
    W = O.hybrid_weights_vec(Y, M, f)
    n_bypass = int((f < 200).sum())
    n_ds = int(np.isclose(np.abs(W[f >= 200, 0]), 0.5, atol=1e-9).sum())
    assert n_bypass == 13                      # 0 .. 187.5 Hz at 15.625 Hz spacing
    assert 0 < n_ds < len(f) - n_bypass        # both branches exercised


def test_singular_noise_covariance_falls_back():
    """No noise-weighted frames: R = 0, the reference would divide by zero (v_int[0] = 0)
    and np.linalg.cond raises; the restatement (and the kernels) take delay-and-sum."""
    rng = np.random.default_rng(0)
    Y = (rng.standard_normal((2, 5, 8)) + 1j * rng.standard_normal((2, 5, 8))).astype(np.complex64)
    f = np.array([0.0, 250.0, 500.0, 1000.0, 2000.0])
    W = O.hybrid_weights_vec(Y, np.ones((5, 8), np.float32), f)
    vt = np.stack([O.steering_vector_phase_norm(x)[:, 0] for x in f])
    assert np.allclose(W[1:], vt[1:] / 2)
    assert (W[0] == [1, 0]).all()


@pytest.mark.parametrize("trip", ["test", "set2"])
def test_enhance_chunked_matches_reference(trip):
    g = golden(f"hybrid_{trip}.npz")
    mix, t, i = triple_f32(trip)
    out = O.enhance_chunked(mix.T.copy(), lambda c, s, seg: O.chunk_target_mask(t, i, s), bf="vec")
    assert out.shape == g["out"].shape
    assert np.abs(out - g["out"]).max() < 1e-5
    L = min(len(out), len(t))
    assert abs(O.projection_sdr_sir(out[:L], t[:L], i[:L])[1] - g["sir_out"]) < 1e-3


def test_chunk_table_matches_driver_loop():
    import importlib
    fp = importlib.import_module("avz.final_pipeline")
    utt, start, base = fp.chunk_table([131632, 16000, 16001, 32000], 16000)
    assert list(base) == [0, 9, 10, 12]
    assert list(start[:9]) == [c * 16000 for c in range(9)]
    assert list(utt) == [0] * 9 + [1] + [2] * 2 + [3] * 2


def test_mask_features_match_reference(g_test):
    """log-magnitude / IPD features the reference computed for chunk 0 of its driver
    (recorded from TFLiteBeamformer.predict_mask's arguments)."""
    mix, _, _ = triple_f32("test")
    f = O.mask_features(mix[:, :32000])
    assert f.dtype == np.float32
    assert np.array_equal(f[0], g_test["chunk0_logmag"])
    assert np.array_equal(f[1], g_test["chunk0_ipd"])
    ft = O.mask_features(mix[:, :32000], layout="tflite")
    assert ft.shape == (513, 64, 4)
    assert np.array_equal(ft[..., 0], f[0])
    assert ft[0, 0, 3] == 0.0 and ft[-1, 0, 3] == 1.0


@pytest.mark.parametrize("trip", ["test", "set2"])
def test_srp_scan_matches_reference(trip):
    """scripts/debug_srp.py power map, captured from the reference's own run."""
    g = golden(f"srp_{trip}.npz")
    mix, _, _ = triple_f32(trip)
    a, P = O.srp_scan(mix)
    assert np.array_equal(a, g["angles"])
    assert np.abs(P - g["power_db"]).max() < 1e-9
