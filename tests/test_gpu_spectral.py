"""GPU parity of the spectral-domain operator surface (avz_beamform_spectral, avz_istft) and
of the stage exports (avz_mvdr_covariance -> avz_solve_covariance -> avz_apply_istft)
against the reference's own outputs (tests/golden/spectral_*.npz: batch_mvdr of
rt_av_zoom/core/tf_lite_version/inference.py:85-179 and its driver's post-filter +
istft; hybrid_test.npz: hybrid_hard_null_bf of Final_pipeline/src/inference.py:28-98)
and the oracle.

Tolerances: the reference accumulates the batch_mvdr covariance in complex64 and solves
in complex128; the engine accumulates in fp64 from the same complex64 STFT, so S agrees to
~1e-6 of its peak (asserted at 1e-5); iSTFT waveforms to 1e-5 absolute (~1e-4 of peak)."""
import numpy as np
import pytest
import torch

from conftest import golden, hybrid_bin_causes, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu

CASES = ["test_ibm", "test_soft", "set2_soft", "test_singular"]


def dev_t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("name", CASES)
def test_batch_mvdr_dropin_matches_reference(gpu_device, name):
    from avz import spectral
    g = golden(f"spectral_{name}.npz")
    d = spectral.get_all_steering_vectors(g["f_bins"], float(g["angle"]), float(g["d"]),
                                          float(g["c"]))
    assert np.array_equal(d[:, :, 0], g["d_vectors"])
    S = spectral.batch_mvdr(g["Y"], g["mask"], g["f_bins"], d, float(g["sigma"]))
    ref = g["S_out"].astype(np.complex128)
    assert S.shape == ref.shape and S.dtype == np.complex128
    err = np.abs(S - ref).max() / np.abs(ref).max()
    print(f"{name}: max |S - S_ref| / max|S_ref| = {err:.2e}")
    assert err <= 1e-5


def test_batch_fallback_flag_and_weights(gpu_device):
    """The singular case: the engine reports the item-level fallback and every bin carries
    w = [1 / (conj(d0) + 1e-10), 0] (tf_lite_version/inference.py:149-163)."""
    from avz import spectral
    g = golden("spectral_test_singular.npz")
    sb = spectral.SpectralBeamformer("mvdr", max_items=2, sigma=0.0, floor=None)
    Y = dev_t(np.stack([g["Y"], golden("spectral_test_soft.npz")["Y"]]), gpu_device)
    M = dev_t(np.stack([g["mask"], golden("spectral_test_soft.npz")["mask"]]), gpu_device)
    flags = torch.full((2,), 7, dtype=torch.int32, device=gpu_device)
    w = torch.zeros((2, 513, 4), dtype=torch.float32, device=gpu_device)
    sb.beamform(Y, M, fallback=flags, w_out=w)
    assert flags.tolist() == [1, 0]
    wd = w[0].cpu().numpy().astype(np.float64)
    d0 = g["d_vectors"][:, 0]
    w0 = 1.0 / (np.conj(d0) + 1e-10)
    assert np.abs(wd[:, 0] + 1j * wd[:, 1] - w0).max() <= 1e-6
    assert (wd[:, 2:] == 0).all()


@pytest.mark.parametrize("name", ["test_ibm", "set2_soft"])
def test_fused_postfilter_and_istft_match_driver(gpu_device, name):
    """The TFLite chunk driver (inference.py:343-352): batch_mvdr -> S * max(M, 0.05) ->
    istft, with the post-filter fused into the beamformer and avz_istft for the iSTFT."""
    from avz import spectral
    g = golden(f"spectral_{name}.npz")
    sb = spectral.SpectralBeamformer("mvdr", max_items=1, sigma=float(g["sigma"]),
                                     d=float(g["d"]), floor=0.05)
    S = sb.beamform(dev_t(g["Y"], gpu_device)[None], dev_t(g["mask"], gpu_device)[None])
    ref = g["S_out"] * np.maximum(g["mask"], 0.05)
    assert np.abs(S[0].cpu().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()
    out, peak = sb.istft(S)
    x = out[0, :len(g["chunk_out"])].cpu().numpy().astype(np.float64)
    err = np.abs(x - g["chunk_out"]).max()
    print(f"{name}: istft max-abs {err:.2e} (peak {np.abs(g['chunk_out']).max():.3f})")
    assert err <= 1e-5
    assert abs(float(peak[0]) - np.abs(g["chunk_out"]).max()) <= 1e-5


def test_hybrid_dropin_matches_reference_chunk0(gpu_device):
    """spectral.hybrid_hard_null_bf on the reference's own chunk-0 STFT and mask: every bin
    whose S differs from the reference's must be explained by conftest.hybrid_bin_causes
    (near-degenerate eigenvector, or the cond_2 branch decided the other way: S then equals
    w_alt^H Y of the other branch). The mask is the reference's, so no count differences."""
    from avz import spectral
    g = golden("hybrid_test.npz")
    Y, M, f = g["chunk0_Y"], g["chunk0_mask"], g["chunk0_f"]
    S = spectral.hybrid_hard_null_bf(Y, M, f)
    ref = g["chunk0_S"].astype(np.complex128)
    tol = 1e-5 * np.abs(ref).max()
    close = np.abs(S - ref).max(axis=1) <= tol
    Yd = Y.astype(np.complex128)

    def matches(k, w):
        return np.abs(S[k] - (w.conj()[0] * Yd[0, k] + w.conj()[1] * Yd[1, k])).max() <= tol

    causes = hybrid_bin_causes(Y, M, f, np.nonzero(~close)[0], matches)
    print(f"hybrid drop-in: {int((~close).sum())} of {len(close)} bins differ: {causes}")
    byp = f < 200.0
    assert np.array_equal(S[byp], Y[0][byp].astype(np.complex128))  # mic 0 passes


def test_batched_items_equal_single_calls(gpu_device):
    from avz import spectral
    names = ["test_ibm", "test_soft", "set2_soft"]
    gs = [golden(f"spectral_{n}.npz") for n in names]
    sb = spectral.SpectralBeamformer("mvdr", max_items=3)
    Y = dev_t(np.stack([g["Y"] for g in gs]), gpu_device)
    M = dev_t(np.stack([g["mask"] for g in gs]), gpu_device)
    S = sb.beamform(Y, M).clone()
    for b in range(3):
        S1 = sb.beamform(Y[b:b + 1].contiguous(), M[b:b + 1].contiguous())
        assert torch.equal(S1[0], S[b])
    # strided (non-contiguous batch) views take the same path
    Yp = torch.zeros((3, 2, 513, 80), dtype=torch.complex64, device=gpu_device)
    Yp[..., :64] = Y
    Mp = torch.zeros((3, 513, 72), dtype=torch.float32, device=gpu_device)
    Mp[..., :64] = M
    S2 = sb.beamform(Yp[..., :64], Mp[..., :64])
    assert torch.equal(S2, S)


@pytest.mark.parametrize("n_fft,T", [(1024, 64), (1024, 37), (512, 126), (512, 9)])
def test_istft_matches_oracle(gpu_device, n_fft, T):
    import avz
    rng = np.random.default_rng(n_fft + T)
    F = n_fft // 2 + 1
    S = (rng.standard_normal((2, F, T)) + 1j * rng.standard_normal((2, F, T))).astype(np.complex64)
    plan = avz.MVDRPlan(n_fft=n_fft, mask="external", postfilter="none", normalize="none",
                        max_batch=2, max_samples=(T - 1) * n_fft // 2)
    out, peak = plan.istft(dev_t(S, gpu_device))
    for b in range(2):
        _, ref = O.istft(S[b].astype(np.complex128), nperseg=n_fft, noverlap=n_fft // 2)
        got = out[b, :len(ref)].cpu().numpy().astype(np.float64)
        assert len(ref) == (T - 1) * n_fft // 2
        assert np.abs(got - ref).max() <= 2e-6 * np.abs(ref).max()
        assert abs(float(peak[b]) - np.abs(ref).max()) <= 2e-6 * np.abs(ref).max()


@pytest.mark.parametrize("n_fft", [512, 1024])
def test_stagewise_chain_equals_fused(gpu_device, n_fft):
    """avz_mvdr_covariance -> avz_solve_covariance -> avz_apply_istft reproduces the fused
    avz_mvdr_batch (oracle IBM mask, no post-filter) and the oracle's R and w."""
    import avz
    mix, t, i = triple_f32("test", seg=(40000, 64000))
    d = gpu_device
    plan = avz.MVDRPlan(n_fft=n_fft, sigma=1e-5, mic_d=0.01, mask="ibm", postfilter="none",
                        normalize="peak", max_batch=1, max_samples=24000)
    m, tt, ii = dev_t(mix, d)[None], dev_t(t, d)[None], dev_t(i, d)[None]
    w_f = torch.zeros((1, plan.F, 4), dtype=torch.float32, device=d)
    out_f, peak_f = plan.run(m, ref_tgt=tt, ref_int=ii, w_out=w_f)
    cov = plan.covariance(m, ref_tgt=tt, ref_int=ii)
    w = plan.solve_covariance(cov)
    assert torch.equal(w, w_f)
    out_s, peak_s = plan.apply_istft(m, w)
    n = plan.out_len(24000)
    assert torch.max(torch.abs(out_s[:, :n] - out_f[:, :n])).item() <= 1e-6
    # against the oracle's stages (oracle_debug.py:56-79)
    f, _, Y = O.stft(mix, nperseg=n_fft, noverlap=n_fft // 2)
    _, _, St = O.stft(t, nperseg=n_fft, noverlap=n_fft // 2)
    _, _, Si = O.stft(i, nperseg=n_fft, noverlap=n_fft // 2)
    mn = O.ibm_mask_noise(St, Si)
    R = O.covariance_vec(Y, mn)
    c = cov[0].cpu().numpy()
    nrm = c[:, 4] + 1e-6
    Rg = np.stack([c[:, 0], c[:, 2] + 1j * c[:, 3], c[:, 2] - 1j * c[:, 3], c[:, 1]], 1) / nrm[:, None]
    assert np.abs(Rg - R.reshape(-1, 4)).max() <= 1e-5 * np.abs(R).max()
    W = O.mvdr_weights_vec(R, f, 1e-5, 90.0, 0.01, 343.0)
    wg = w[0].cpu().numpy().astype(np.float64)
    Wg = np.stack([wg[:, 0] + 1j * wg[:, 1], wg[:, 2] + 1j * wg[:, 3]], 1)
    assert np.abs(Wg - W).max() <= 1e-3 * np.abs(W).max()


def test_apply_istft_gain_equals_ibm_postfilter(gpu_device):
    """avz_apply_istft with gain = 1 - mask_noise (the IBM post-filter as an external gain)
    equals the fused IBM chain with its post-filter."""
    import avz
    mix, t, i = triple_f32("set2", seg=(10000, 42000))
    d = gpu_device
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=1, max_samples=32000)
    m, tt, ii = dev_t(mix, d)[None], dev_t(t, d)[None], dev_t(i, d)[None]
    w_f = torch.zeros((1, plan.F, 4), dtype=torch.float32, device=d)
    out_f, _ = plan.run(m, ref_tgt=tt, ref_int=ii, w_out=w_f)
    Yr = plan.stft(torch.stack([tt, ii], 1))[0]                  # [2, F, T]
    gain = (torch.abs(Yr[1]) <= torch.abs(Yr[0])).float()[None]   # 1 - (|S_int| > |S_tgt|)
    out_s, _ = plan.apply_istft(m, w_f, gain=gain.contiguous())
    n = plan.out_len(32000)
    assert torch.max(torch.abs(out_s[:, :n] - out_f[:, :n])).item() <= 2e-4


@pytest.mark.parametrize("T", [37, 64, 100])
def test_batch_mvdr_frame_counts_vs_oracle(gpu_device, T):
    """Both spectral layouts: <= 64 frames (16 lanes per row, frames in registers) and
    longer spectra (one wave per row); random complex64 Y and a uniform mask, against the
    oracle's batch_mvdr (tf_lite_version/inference.py:85-179 restated)."""
    from avz import spectral
    rng = np.random.default_rng(T)
    F = 513
    Y = (rng.standard_normal((2, F, T)) + 1j * rng.standard_normal((2, F, T))).astype(np.complex64)
    M = rng.random((F, T)).astype(np.float32)
    f_bins = np.fft.rfftfreq(1024, 1 / 16000)
    d = spectral.get_all_steering_vectors(f_bins, 90.0, 0.04, 343.0)
    ref = O.batch_mvdr(Y, M, f_bins, d, 1e-5)
    S = spectral.batch_mvdr(Y, M, f_bins, d, 1e-5)
    err = np.abs(S - ref).max() / np.abs(ref).max()
    assert err <= 1e-5, err
