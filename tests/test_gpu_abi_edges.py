"""GPU: edge behaviour of the C ABI.

- a NaN in one bin's STFT under batch_mvdr semantics (AVZ_FALLBACK_BATCH) gives NaN in
  that bin only, as the reference's np.linalg.solve does (LAPACK raises only on an exactly
  zero pivot, so there is no item-level fallback): checked against the oracle's batch_mvdr
  (tf_lite_version/inference.py:85-179 restated); parity unpinned by a reference-run
  fixture (none of the reference's own files holds a NaN input);
- misaligned device pointers are rejected with AVZ_ERR_ALIGN before any launch;
- the covariance stage (avz_mvdr_covariance) leaves the caller's out / peak untouched."""
import ctypes as ct

import numpy as np
import pytest
import torch

from conftest import golden, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu


def dev_t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_nan_bin_propagates_under_batch_fallback(gpu_device):
    from avz import spectral
    g = golden("spectral_test_soft.npz")
    Y = g["Y"].copy()
    Y[0, 100, 5] = np.nan
    sb = spectral.SpectralBeamformer("mvdr", max_items=2, sigma=float(g["sigma"]), floor=None)
    flags = torch.full((2,), 7, dtype=torch.int32, device=gpu_device)
    S = sb.beamform(dev_t(np.stack([g["Y"], Y]), gpu_device),
                    dev_t(np.stack([g["mask"], g["mask"]]), gpu_device), fallback=flags)
    S = S.cpu().numpy()
    assert flags.tolist() == [0, 0]
    nan_bins = np.nonzero(np.isnan(S[1]).any(axis=1))[0]
    assert nan_bins.tolist() == [100] and np.isnan(S[1, 100]).all()
    keep = np.arange(S.shape[1]) != 100
    assert np.array_equal(S[1, keep], S[0, keep])
    d = O.get_all_steering_vectors(g["f_bins"], float(g["angle"]), float(g["d"]), float(g["c"]))
    with np.errstate(invalid="ignore"):
        ref = O.batch_mvdr(Y, g["mask"], g["f_bins"], d, float(g["sigma"]))
    assert np.array_equal(np.isnan(ref), np.isnan(S[1]))


def test_misaligned_pointers_rejected(gpu_device):
    import avz
    from avz._lib import AVZ_ERR_ALIGN, AvzSpectralArgs, lib
    plan = avz.MVDRPlan(n_fft=1024, mask="external", postfilter="none", normalize="none",
                        weight_eps=1e-10, fmin_hz=0.0, singular_fallback="batch",
                        max_batch=1, max_samples=32256)
    F, T = 513, 64
    raw = torch.zeros(2 * F * T * 2 + 64, dtype=torch.float32, device=gpu_device)
    mask = torch.zeros(F * T + 64, dtype=torch.float32, device=gpu_device)
    S = torch.zeros(F * T * 2 + 64, dtype=torch.float32, device=gpu_device)
    base = raw.data_ptr()

    def spectral(y_off, m_off, s_off):
        a = AvzSpectralArgs()
        a.batch, a.frames = 1, T
        a.Y = base + y_off
        a.y_stride_b, a.y_stride_m, a.y_stride_f = 2 * F * T, F * T, T
        a.mask = mask.data_ptr() + m_off
        a.mask_stride_b, a.mask_stride_f = F * T, T
        a.S = S.data_ptr() + s_off
        a.s_stride_b, a.s_stride_f = F * T, T
        return lib.avz_beamform_spectral(plan._h, ct.byref(a), None)

    assert spectral(0, 0, 0) == 0
    assert spectral(4, 0, 0) == AVZ_ERR_ALIGN
    assert spectral(0, 0, 4) == AVZ_ERR_ALIGN
    assert spectral(0, 2, 0) == AVZ_ERR_ALIGN
    out = torch.zeros((1, 32256 + 64), dtype=torch.float32, device=gpu_device)
    assert lib.avz_istft(plan._h, 1, T, ct.c_void_p(S.data_ptr() + 4), F * T, T,
                         ct.c_void_p(out.data_ptr()), out.stride(0), None, None, 0,
                         None) == AVZ_ERR_ALIGN
    cov = torch.zeros(F * 5 + 8, dtype=torch.float64, device=gpu_device)
    w = torch.zeros(F * 4 + 8, dtype=torch.float32, device=gpu_device)
    assert lib.avz_solve_covariance(plan._h, 1, ct.c_void_p(cov.data_ptr() + 4),
                                    ct.c_void_p(w.data_ptr()), None, None, None) == AVZ_ERR_ALIGN
    assert lib.avz_solve_covariance(plan._h, 1, ct.c_void_p(cov.data_ptr()),
                                    ct.c_void_p(w.data_ptr() + 8), None, None, None) == AVZ_ERR_ALIGN
    torch.cuda.synchronize()


def test_covariance_stage_leaves_out_and_peak(gpu_device):
    import avz
    from avz._lib import lib
    mix, t, i = triple_f32("test", seg=(0, 24000))
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="none", max_batch=1, max_samples=24000)
    m, tt, ii = dev_t(mix, gpu_device)[None], dev_t(t, gpu_device)[None], dev_t(i, gpu_device)[None]
    out = torch.full((1, plan.out_len(24000) + 4), 3.0, device=gpu_device)
    peak = torch.full((1,), 7.0, device=gpu_device)
    cov = torch.zeros((1, plan.F, 5), dtype=torch.float64, device=gpu_device)
    a, _, _ = plan._batch_args(m, None, None, tt, ii, None, out, peak, cov, None, None)
    assert a.peak == peak.data_ptr() and a.out == out.data_ptr()
    assert lib.avz_mvdr_covariance(plan._h, ct.byref(a), None) == 0
    torch.cuda.synchronize()
    assert float(peak[0]) == 7.0 and bool((out == 3.0).all())
    assert torch.equal(cov, plan.covariance(m, ref_tgt=tt, ref_int=ii))
