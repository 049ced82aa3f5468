"""GPU: mask-model input features (avz_mask_features) against the features the
reference computed inside its Final_pipeline driver (chunk 0 of the test triple,
tests/golden/hybrid_test.npz) and against the oracle for the TFLite NHWC layout.

Tolerance: the GPU STFT is fp32 (scipy's is fp64 rounded to complex64), so |Y| agrees to
~2e-6 of max|Y|; log(|Y|+1e-7) and angles are compared with that error propagated
(d log = d|Y| / (|Y|+1e-7), d angle = d|Y| / |Y|). An angle near the negative real axis
can land on the other side of the branch cut (a 2 pi jump); those are counted and must be
such near-cut bins."""
import numpy as np
import pytest
import torch

from conftest import golden, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def feats(gpu_device):
    import avz
    from avz.engine import mask_features
    mix, _, _ = triple_f32("test")
    x = torch.from_numpy(np.ascontiguousarray(mix[:, :32000]))[None].to(gpu_device)
    plan = avz.MVDRPlan(n_fft=1024, mask="external", postfilter="mul", max_batch=1,
                        max_samples=32000)
    u = mask_features(plan, x, "unet")[0].cpu().numpy()
    t = mask_features(plan, x, "tflite")[0].cpu().numpy()
    _, _, Y = O.stft(mix[:, :32000], nperseg=1024, noverlap=512)
    return u, t, Y


def _check(got_lm, got_ipd, ref_lm, ref_ipd, Y):
    amax = np.abs(Y).max()
    d_abs = 4e-6 * amax
    tol_lm = d_abs / (np.abs(Y[0]) + 1e-7) + 1e-5
    assert (np.abs(got_lm - ref_lm) <= tol_lm).all()
    d = got_ipd - ref_ipd
    wrapped = np.abs(np.abs(d) - 2 * np.pi) < 1e-3
    tol = d_abs / np.minimum(np.abs(Y[0]), np.abs(Y[1])).clip(1e-30) + 1e-5
    ok = (np.abs(d) <= tol) | wrapped
    assert ok.all()
    # every 2 pi jump sits on the branch cut (imaginary part within rounding of zero)
    if wrapped.any():
        near = (np.abs(Y[0].imag) <= d_abs) | (np.abs(Y[1].imag) <= d_abs)
        assert near[wrapped].all()
    return int(wrapped.sum())


def test_unet_features_vs_reference(feats):
    u, _, Y = feats
    g = golden("hybrid_test.npz")
    assert u.shape == (2, 513, 64)
    _check(u[0], u[1], g["chunk0_logmag"], g["chunk0_ipd"], Y)


def test_tflite_features_vs_oracle(feats):
    u, t, Y = feats
    mix, _, _ = triple_f32("test")
    ref = O.mask_features(mix[:, :32000], layout="tflite")
    assert t.shape == ref.shape == (513, 64, 4)
    assert np.array_equal(t[..., 0], u[0])
    ipd = u[1]
    assert np.allclose(t[..., 1], np.sin(ipd), atol=2e-6)
    assert np.allclose(t[..., 2], np.cos(ipd), atol=2e-6)
    assert np.array_equal(t[..., 3], ref[..., 3])


def test_srp_scan_vs_reference(gpu_device):
    """Batched SRP scan (avz_srp_scan) of both bundled mixtures in one call against the
    power maps the reference's scripts/debug_srp.py computed (0.07-0.09 dB dynamic range
    at d = 0.01 m, so the tolerance is absolute: 1e-4 dB)."""
    import avz
    from avz.engine import srp_scan
    trips = ["test", "set2"]
    mixes = [triple_f32(k)[0] for k in trips]
    S = max(m.shape[1] for m in mixes)
    x = np.zeros((2, 2, S), np.float32)
    for b, m in enumerate(mixes):
        x[b, :, :m.shape[1]] = m
    lens = torch.tensor([m.shape[1] for m in mixes], dtype=torch.int32, device=gpu_device)
    plan = avz.MVDRPlan(n_fft=512, mic_d=0.01, mask="ones", postfilter="none", max_batch=2,
                        max_samples=S)
    P = srp_scan(plan, torch.from_numpy(x).to(gpu_device), lens, max_len=S).cpu().numpy()
    for b, k in enumerate(trips):
        g = golden(f"srp_{k}.npz")
        assert np.abs(P[b] - g["power_db"]).max() < 1e-4
        assert P[b].argmax() == g["power_db"].argmax()
