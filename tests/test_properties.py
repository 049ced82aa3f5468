"""Property tests of the CPU restatement (hypothesis): scipy-exact framing and perfect
reconstruction for arbitrary lengths, and the closed-form 2x2 solves against LAPACK.
CPU only; these are the properties the GPU tests then check at full size."""
import numpy as np
import scipy.signal
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import avz_oracle as O


@settings(max_examples=25, deadline=None)
@given(n=st.sampled_from([512, 1024]), length=st.integers(min_value=1024, max_value=9000),
       seed=st.integers(0, 2**31 - 1))
def test_stft_istft_round_trip(n, length, seed):
    """scipy.signal.stft -> istft is a perfect reconstruction at 50 % Hann overlap: the
    restatement's output equals the input on its length (extra tail samples are the
    zero padding), and its frame count is ceil(L / hop) + 1."""
    x = np.random.default_rng(seed).standard_normal(length).astype(np.float32)
    _, _, Y = O.stft(x, nperseg=n, noverlap=n // 2)
    assert Y.shape == (n // 2 + 1, O.n_frames(length, n, n // 2))
    assert Y.shape[1] == -(-length // (n // 2)) + 1
    _, xr = O.istft(Y, nperseg=n, noverlap=n // 2)
    assert len(xr) == (Y.shape[1] - 1) * (n // 2) >= length
    np.testing.assert_allclose(xr[:length], x, atol=2e-6)
    np.testing.assert_allclose(xr[length:], 0.0, atol=2e-6)
    _, _, Ys = scipy.signal.stft(x, fs=16000, nperseg=n, noverlap=n // 2)
    assert np.max(np.abs(Ys - Y)) <= 1e-6 * np.max(np.abs(Ys))


def _hermitian_pd(rng, nb, scale):
    a = rng.standard_normal((nb, 2, 2)) + 1j * rng.standard_normal((nb, 2, 2))
    return scale * (a @ np.conj(np.transpose(a, (0, 2, 1))))


@settings(max_examples=20, deadline=None)
@given(seed=st.integers(0, 2**31 - 1), sigma=st.sampled_from([1.0, 1e-3, 1e-5, 1e-7]),
       scale=st.sampled_from([1e-8, 1e-4, 1.0]))
def test_closed_form_mvdr_matches_lapack(seed, sigma, scale):
    """The closed-form 2x2 Hermitian solve the kernels use (oracle mvdr_weights_vec)
    equals the reference's per-bin np.linalg.solve loop (oracle_debug.py:66-79)."""
    rng = np.random.default_rng(seed)
    R = _hermitian_pd(rng, 64, scale)
    f = np.fft.rfftfreq(126, 1 / 16000)[:64]
    Wl = O.mvdr_weights_loop(R, f, sigma, 90.0, 0.01, 343.0)
    Wv = O.mvdr_weights_vec(R, f, sigma, 90.0, 0.01, 343.0)
    np.testing.assert_allclose(Wv, Wl, rtol=1e-8, atol=1e-12 * np.max(np.abs(Wl)))


@settings(max_examples=20, deadline=None)
@given(seed=st.integers(0, 2**31 - 1))
def test_mvdr_distortionless(seed):
    """MVDR weights satisfy w^H d = 1 up to the reference's +1e-10 (f >= fmin)."""
    rng = np.random.default_rng(seed)
    R = _hermitian_pd(rng, 40, 1.0)
    f = np.linspace(100.0, 8000.0, 40)
    W = O.mvdr_weights_vec(R, f, 1e-3, 90.0, 0.04, 343.0)
    d = O.steering_vectors(f, 90.0, 0.04, 343.0)
    resp = np.sum(np.conj(W) * d, axis=1)
    np.testing.assert_allclose(resp, 1.0, atol=1e-8)


@settings(max_examples=20, deadline=None)
@given(seed=st.integers(0, 2**31 - 1))
def test_hybrid_closed_form_matches_loop(seed):
    """The hybrid hard-null closed form (eigenvector, cond test, (C^H)^-1 e1) equals the
    reference-faithful loop (Final_pipeline/src/inference.py:28-98) on random chunks."""
    rng = np.random.default_rng(seed)
    F, T = 40, 24
    Y = (rng.standard_normal((2, F, T)) + 1j * rng.standard_normal((2, F, T))).astype(np.complex64)
    mask = (rng.random((F, T)) > 0.5).astype(np.float32)
    f = np.linspace(0.0, 8000.0, F)
    Wl = O.hybrid_weights_loop(Y, mask, f)
    Wv = O.hybrid_weights_vec(Y, mask, f)
    np.testing.assert_allclose(Wv, Wl, rtol=1e-5, atol=1e-5 * np.max(np.abs(Wl)))
