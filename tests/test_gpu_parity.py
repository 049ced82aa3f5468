"""GPU parity: the HIP path (through the C ABI) against the pinned CPU oracle and the
reference's golden vectors. Tolerances (BASELINE.md section 4 / SURVEY 8(a)):
peak-normalised waveform max-abs <= 1e-4 and SIR |delta| <= 0.01 dB vs the reference
on identical inputs; STFT bins within 2e-6 of max|Y| (fp32 FFT vs pocketfft)."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu

WAVE_TOL = 1e-4
SIR_TOL = 0.01


@pytest.fixture(scope="module")
def avz(gpu_device):
    import avz as _avz
    return _avz


def dev_t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def run_ibm(avz, dev, mix, tgt, itf, n, sigma, normalize="peak", debug=False, mic_d=0.01):
    plan = avz.MVDRPlan(n_fft=n, sigma=sigma, mic_d=mic_d, mask="ibm", postfilter="ibm",
                        normalize=normalize, max_batch=1, max_samples=len(tgt))
    F = n // 2 + 1
    cov = torch.zeros((1, F, 5), dtype=torch.float64, device=dev) if debug else None
    w = torch.zeros((1, F, 4), dtype=torch.float32, device=dev) if debug else None
    out, peak = plan.run(dev_t(mix, dev)[None], ref_tgt=dev_t(tgt, dev)[None],
                         ref_int=dev_t(itf, dev)[None], cov_out=cov, w_out=w)
    torch.cuda.synchronize()
    n_out = plan.out_len(len(tgt))
    res = out[0, :n_out].cpu().numpy().astype(np.float64)
    if debug:
        return res, float(peak[0]), cov[0].cpu().numpy(), w[0].cpu().numpy()
    return res, float(peak[0])


def sir(out, tgt, itf):
    L = min(len(out), len(tgt))
    return O.projection_sdr_sir(out[:L], tgt[:L], itf[:L])[1]


# ----------------------------------------------------------------------------- STFT stage
@pytest.mark.parametrize("n", [512, 1024])
def test_stft_stage(avz, gpu_device, n):
    rng = np.random.default_rng(n)
    lens = [n, n + 1, 3 * n // 2 + 7, 20000]
    S = max(lens)
    x = np.zeros((len(lens), 2, S), np.float32)
    for b, L in enumerate(lens):
        x[b, :, :L] = rng.standard_normal((2, L)).astype(np.float32)
    plan = avz.MVDRPlan(n_fft=n, mask="ipd", postfilter="none", max_batch=len(lens), max_samples=S)
    Y = plan.stft(dev_t(x, gpu_device), torch.tensor(lens, dtype=torch.int32, device=gpu_device),
                  max_len=S).cpu().numpy()
    for b, L in enumerate(lens):
        _, _, Yr = O.stft(x[b, :, :L], nperseg=n, noverlap=n // 2)
        T = Yr.shape[-1]
        got = Y[b, :, :, :T]
        assert np.max(np.abs(got - Yr)) <= 2e-6 * np.max(np.abs(Yr))
        # DC / Nyquist imaginary parts are exactly +0 (pocketfft r2c)
        assert np.all(got[:, 0, :].imag == 0) and np.all(got[:, -1, :].imag == 0)
        assert not np.any(np.signbit(got[:, 0, :].imag))


# ----------------------------------------------------------------------------- fused IBM
MAX_IBM_FLIPS = 0      # exact decisions (avz_ibm_exact.hpp); 0-2 ties per golden before round 6
IBM_TIE_MARGIN = 1e-7  # fp32 FFT rounding relative to the frame's largest bin; measured <= 1.6e-8


def ibm_flip_report(name, cov, st):
    """Mask fidelity of the IBM chain: per-bin noise-frame counts (cov_out column 4) against
    the oracle's (pinned to the reference's stage_* goldens). Counts are exact except where
    |S_int| ~ |S_tgt| to within fp32 FFT rounding (the GPU STFT is fp32; scipy's is fp64
    rounded to complex64). FFT error scales with the frame's largest bin, so every flipped
    (bin, frame) must be a tie relative to that scale: a bin's count may move by at most its
    number of tie frames (|d| < IBM_TIE_MARGIN of the scale), and a golden holds at most
    MAX_IBM_FLIPS flips in all."""
    msum = st["mask"].sum(axis=1)
    diff = np.nonzero(cov[:, 4] != msum)[0]
    frame_scale = np.maximum(np.abs(st["S_i"]).max(axis=0), np.abs(st["S_t"]).max(axis=0))
    margins = []
    for k in diff:
        a, b = np.abs(st["S_i"][k]), np.abs(st["S_t"][k])
        rel = np.abs(a - b) / np.maximum(frame_scale, 1e-30)
        n_ties = int(np.sum(rel < IBM_TIE_MARGIN))
        margins.append(float(np.min(rel)))
        assert abs(cov[k, 4] - msum[k]) <= n_ties, (k, cov[k, 4], msum[k], np.min(rel))
    n_flip = int(np.sum(np.abs(cov[diff, 4] - msum[diff])))
    print(f"{name}: IBM flips {n_flip} in {len(diff)}/{len(msum)} bins "
          f"(all ties; max relative margin {max(margins, default=0.0):.1e}), non-tie flips 0")
    assert n_flip <= MAX_IBM_FLIPS, n_flip


EXC = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "excerpt_*.npz")))
FULL = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "full_*.npz")))


@pytest.mark.parametrize("name", EXC)
def test_fused_ibm_excerpt_vs_reference(avz, gpu_device, name):
    g = golden(name)
    trip = name.split("_")[1]
    mix, tgt, itf = triple_f32(trip, g["seg"])
    n, s = int(g["n_fft"]), float(g["sigma"])
    out, peak, cov, w = run_ibm(avz, gpu_device, mix, tgt, itf, n, s, debug=True)
    ref = g["out"].astype(np.float64)
    assert len(out) == len(ref)
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - sir(ref, tgt, itf)) <= SIR_TOL
    assert abs(peak - float(g["peak_raw"])) <= 1e-4 * float(g["peak_raw"])
    # stage parity against the oracle's fp64 covariance / weights
    _, st = O.oracle_debug_vec(mix, tgt, itf, n_fft=n, hop=n // 2, sigma=s, return_stages=True)
    ibm_flip_report(name, cov, st)
    msum = st["mask"].sum(axis=1)
    ok = cov[:, 4] == msum
    R = st["R"] * (msum + 1e-6)[:, None, None]
    scale = np.max(np.abs(R[:, 0, 0]))
    np.testing.assert_allclose(cov[ok, 0], R[ok, 0, 0].real, atol=2e-6 * scale)
    np.testing.assert_allclose(cov[ok, 2] + 1j * cov[ok, 3], R[ok, 0, 1], atol=2e-6 * scale)
    W = w[:, 0] + 1j * w[:, 1], w[:, 2] + 1j * w[:, 3]
    np.testing.assert_allclose(W[0][ok], st["W"][ok, 0], atol=1e-3 * np.max(np.abs(st["W"])))
    np.testing.assert_allclose(W[1][ok], st["W"][ok, 1], atol=1e-3 * np.max(np.abs(st["W"])))


@pytest.mark.parametrize("n", [512, 1024])
def test_fused_solve_full_batch_vs_reference(avz, gpu_device, n):
    """The headline's kernels on a reference-run fixture: a batch of #CU copies of the
    bundled test triple (one whole utterance per per-utterance synthesis block, the block
    solving its utterance's bins itself, no piece split) against full_test_n{n}_s1 (the
    reference's oracle_debug.main output); the same batch with the covariance / weight debug
    outputs (solve kernel, unfused) must be bitwise equal (bin_cov_sums_utt sums as
    bin_cov_sums does), and every copy equal to the first."""
    g = golden(f"full_test_n{n}_s1.npz")
    mix, tgt, itf = triple_f32("test")
    B = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    S = len(tgt)
    plan = avz.MVDRPlan(n_fft=n, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=B, max_samples=S)
    dm = dev_t(mix, gpu_device)[None].expand(B, -1, -1).contiguous()
    dt = dev_t(tgt, gpu_device)[None].expand(B, -1).contiguous()
    di = dev_t(itf, gpu_device)[None].expand(B, -1).contiguous()
    out, peak = plan.run(dm, ref_tgt=dt, ref_int=di)
    out, peak = out.clone(), peak.clone()
    F = n // 2 + 1
    cov = torch.zeros((B, F, 5), dtype=torch.float64, device=gpu_device)
    w = torch.zeros((B, F, 4), dtype=torch.float32, device=gpu_device)
    out_d, peak_d = plan.run(dm, ref_tgt=dt, ref_int=di, cov_out=cov, w_out=w)
    torch.cuda.synchronize()
    n_out = plan.out_len(S)
    assert torch.equal(out[:, :n_out], out_d[:, :n_out]) and torch.equal(peak, peak_d)
    assert torch.equal(out[:, :n_out], out[:1, :n_out].expand(B, -1))
    res = out[0, :n_out].cpu().numpy().astype(np.float64)
    assert len(res) == int(g["out_len"])
    assert np.max(np.abs(res[::16] - g["out_stride16"])) <= WAVE_TOL
    assert np.max(np.abs(res[:4096] - g["out_head"])) <= WAVE_TOL
    assert abs(sir(res, tgt, itf) - float(g["sir_out"])) <= SIR_TOL
    assert abs(float(peak[0]) - float(g["peak_raw"])) <= 1e-4 * float(g["peak_raw"])


@pytest.mark.parametrize("name", FULL)
def test_fused_ibm_full_length_vs_reference(avz, gpu_device, name):
    g = golden(name)
    trip = name.split("_")[1]
    mix, tgt, itf = triple_f32(trip)
    n, s = int(g["n_fft"]), float(g["sigma"])
    out, _, cov, _ = run_ibm(avz, gpu_device, mix, tgt, itf, n, s, debug=True)
    assert len(out) == int(g["out_len"])
    assert np.max(np.abs(out[::16] - g["out_stride16"])) <= WAVE_TOL
    assert np.max(np.abs(out[:4096] - g["out_head"])) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - float(g["sir_out"])) <= SIR_TOL
    # full-array check against the oracle (identical inputs)
    ref, st = O.oracle_debug_vec(mix, tgt, itf, n_fft=n, hop=n // 2, sigma=s, return_stages=True)
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    ibm_flip_report(name, cov, st)


# ----------------------------------------------------------------------------- fused IPD
@pytest.mark.parametrize("trip", ["test", "set2"])
@pytest.mark.parametrize("n", [512, 1024])
def test_fused_ipd_vs_reference(avz, gpu_device, trip, n):
    g = golden(f"ipd_{trip}_n{n}.npz")
    mix, tgt, itf = triple_f32(trip)
    plan = avz.MVDRPlan(n_fft=n, sigma=1e-7, mic_d=0.01, mask="ipd", postfilter="none",
                        normalize="peak", norm_eps=1e-6, max_batch=1, max_samples=len(tgt))
    F = n // 2 + 1
    cov = torch.zeros((1, F, 5), dtype=torch.float64, device=gpu_device)
    out, _ = plan.run(dev_t(mix, gpu_device)[None], cov_out=cov)
    torch.cuda.synchronize()
    out = out[0, :plan.out_len(len(tgt))].cpu().numpy().astype(np.float64)
    assert len(out) == int(g["out_len"])
    ref, st = O.masked_mvdr_vec(mix, n_fft=n, hop=n // 2, return_stages=True)
    # mask fidelity: per-bin weight sums (1 or 0.01 per frame) against the reference's;
    # a (bin, frame) decided differently moves its bin's sum by 0.99
    msum = cov[0, :, 4].cpu().numpy()
    rsum = st["mask"].astype(np.float64).sum(axis=1)
    dev = np.abs(msum - rsum)
    n_dev = int(np.sum(np.round(dev / 0.99)))
    print(f"ipd_{trip}_n{n}: IPD mask decisions differing from the reference: {n_dev} of "
          f"{st['mask'].size} (max |sum diff| {dev.max():.2e})")
    assert n_dev == 0
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    assert np.max(np.abs(out[::16] - g["out_stride16"])) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - float(g["sir_out"])) <= SIR_TOL


# ----------------------------------------------------------------------------- external mask
@pytest.mark.parametrize("n", [512, 1024])
@pytest.mark.parametrize("floor", [0.05, None])
def test_fused_external_mask(avz, gpu_device, n, floor):
    mix, tgt, itf = triple_f32("set2", (10000, 42000))
    _, _, S_t = O.stft(tgt, nperseg=n, noverlap=n // 2)
    _, _, S_i = O.stft(itf, nperseg=n, noverlap=n // 2)
    rng = np.random.default_rng(3)
    # a soft "neural" target probability: IRM-like plus noise, clipped to [0, 1]
    M = np.abs(S_t) ** 2 / (np.abs(S_t) ** 2 + np.abs(S_i) ** 2 + 1e-10)
    M = np.clip(M + 0.1 * rng.standard_normal(M.shape), 0, 1).astype(np.float32)
    ref = O.external_mask_vec(mix, M, n_fft=n, hop=n // 2, sigma=1e-5, d=0.04, floor=floor)
    plan = avz.MVDRPlan(n_fft=n, sigma=1e-5, mic_d=0.04, mask="external",
                        postfilter="floor" if floor is not None else "none",
                        pf_floor=floor or 0.0, normalize="none", max_batch=1,
                        max_samples=len(tgt))
    out, peak = plan.run(dev_t(mix, gpu_device)[None], ext_mask=dev_t(M, gpu_device)[None])
    torch.cuda.synchronize()
    got = out[0, :len(ref)].cpu().numpy()
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(got - ref)) <= WAVE_TOL * scale
    assert abs(float(peak[0]) - scale) <= 1e-4 * scale
    # the same mask as a transposed (bin-contiguous) view: the kernels' strided path
    Mt = dev_t(np.ascontiguousarray(M.T), gpu_device).t()
    out2, _ = plan.run(dev_t(mix, gpu_device)[None], ext_mask=Mt[None])
    torch.cuda.synchronize()
    got2 = out2[0, :len(ref)].cpu().numpy()
    assert np.max(np.abs(got2 - ref)) <= WAVE_TOL * scale
    # t-contiguous rows padded to a multiple of 4 frames (16-B aligned row starts) while T
    # itself is not: 16-B row-segment reads on the full steps, scalar reads on the last
    T = M.shape[1]
    Mp = np.zeros((M.shape[0], -(-T // 4) * 4), np.float32)
    Mp[:, :T] = M
    out3, _ = plan.run(dev_t(mix, gpu_device)[None], ext_mask=dev_t(Mp, gpu_device)[None, :, :T])
    torch.cuda.synchronize()
    got3 = out3[0, :len(ref)].cpu().numpy()
    assert np.max(np.abs(got3 - ref)) <= WAVE_TOL * scale


# ----------------------------------------------------------------------------- batching
@pytest.mark.parametrize("n", [512, 1024])
def test_batch_ragged_lengths_match_single(avz, gpu_device, n):
    """Variable-length utterances in one launch: each equals the oracle on its own."""
    mix, tgt, itf = triple_f32("test")
    lens = [n, n + 1, 5000, 16001, 64000, 40960]
    S = max(lens)
    offs = [0, 3000, 7000, 11000, 20000, 30000]
    B = len(lens)
    m = np.zeros((B, 2, S), np.float32)
    t = np.zeros((B, S), np.float32)
    i = np.zeros((B, S), np.float32)
    for b, (L, o) in enumerate(zip(lens, offs)):
        m[b, :, :L] = mix[:, o:o + L]
        t[b, :L] = tgt[o:o + L]
        i[b, :L] = itf[o:o + L]
    plan = avz.MVDRPlan(n_fft=n, sigma=1e-5, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=B, max_samples=S)
    out, peak = plan.run(dev_t(m, gpu_device), torch.tensor(lens, dtype=torch.int32,
                                                            device=gpu_device), max_len=S,
                         ref_tgt=dev_t(t, gpu_device), ref_int=dev_t(i, gpu_device))
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    for b, L in enumerate(lens):
        ref = O.oracle_debug_vec(m[b, :, :L], t[b, :L], i[b, :L], n_fft=n, hop=n // 2, sigma=1e-5)
        assert np.max(np.abs(out[b, :len(ref)] - ref)) <= WAVE_TOL, b


def test_plan_rejects_bad_shapes(avz, gpu_device):
    plan = avz.MVDRPlan(n_fft=1024, mask="ibm", postfilter="ibm", max_batch=2, max_samples=4096)
    x = torch.zeros((1, 2, 8192), device=gpu_device)
    with pytest.raises(avz.AvzError):
        plan.run(x, ref_tgt=x[:, 0], ref_int=x[:, 1])        # longer than max_samples
    with pytest.raises(avz.AvzError):
        plan.run(x[:, :, :2048])                             # IBM without references
    with pytest.raises(avz.AvzError):
        avz.MVDRPlan(n_fft=768)


# ----------------------------------------------------------------------------- IPD ties
def test_ipd_identical_channels(avz, gpu_device):
    """Degenerate IPD input: both channels identical, so masked_mvdr.py:37-46 sees
    bitwise-equal angles in every bin and weights them all 0.01. The packed FFT's split
    does not reproduce bitwise-equal channel spectra, so the analysis kernel flags frames
    whose two channels are bitwise identical and gives every bin of them the reference's
    0.01: the per-bin mask sums equal the reference's, and the output the oracle's."""
    mix, tgt, itf = triple_f32("test")
    n = 1024
    mono = np.ascontiguousarray(np.stack([mix[0], mix[0]]))
    plan = avz.MVDRPlan(n_fft=n, sigma=1e-7, mic_d=0.01, mask="ipd", postfilter="none",
                        normalize="peak", norm_eps=1e-6, max_batch=1, max_samples=mono.shape[1])
    F = n // 2 + 1
    cov = torch.zeros((1, F, 5), dtype=torch.float64, device=gpu_device)
    out, _ = plan.run(dev_t(mono, gpu_device)[None], cov_out=cov)
    torch.cuda.synchronize()
    out = out[0, :plan.out_len(mono.shape[1])].cpu().numpy().astype(np.float64)
    ref, st = O.masked_mvdr_vec(mono, n_fft=n, hop=n // 2, return_stages=True)
    # sum of mask weights per bin (cov column 4) vs the reference's
    msum = cov[0, :, 4].cpu().numpy()
    rsum = st["mask"].astype(np.float64).sum(axis=1)
    print(f"identical channels: max |mask sum - ref| = {np.max(np.abs(msum - rsum)):.3g} "
          f"(ref sum per bin {rsum[10]:.3g}), max |out - ref| = {np.max(np.abs(out - ref)):.3g}")
    np.testing.assert_allclose(msum, rsum, rtol=1e-6)
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    # one channel differing in a single sample: only the frames that see it leave the flag;
    # there the two spectra differ by a tiny amount, so bins whose reference angles agree to
    # within fp32 rounding are genuine ties (decided by the last bit of each STFT)
    mono2 = mono.copy()
    mono2[1, 20000] += 1e-3
    out2, _ = plan.run(dev_t(mono2, gpu_device)[None], cov_out=cov)
    torch.cuda.synchronize()
    _, st2 = O.masked_mvdr_vec(mono2, n_fft=n, hop=n // 2, return_stages=True)
    msum2 = cov[0, :, 4].cpu().numpy()
    rsum2 = st2["mask"].astype(np.float64).sum(axis=1)
    dev_bins = np.nonzero(np.round(np.abs(msum2 - rsum2) / 0.99))[0]
    ang = np.angle(st2["Y"].astype(np.complex128))
    dphi = np.abs(np.angle(np.exp(1j * (ang[0] - ang[1]))))  # [F, T]
    for k in dev_bins:
        assert np.min(dphi[k][dphi[k] > 0], initial=0.0) < 1e-6, (k, np.min(dphi[k]))
    print(f"one differing sample: mask decisions differing from the reference: "
          f"{len(dev_bins)} bins, all angle ties (|d angle| < 1e-6 rad)")


@pytest.mark.parametrize("mask,n_fft", [("ibm", 1024), ("ibm", 512), ("ipd", 1024)])
def test_multi_round_ragged_batch_equals_single_runs(avz, gpu_device, mask, n_fft):
    """A batch larger than one pass of the persistent grids (300 utterances against 256
    per-utterance synthesis blocks and 2-3 analysis blocks per CU, so blocks loop over
    several utterances / items of different lengths) with ragged lengths, for both
    per-utterance synthesis kernels (N = 1024, 512) and the IPD plan (no post-filter).
    The partial last rounds are split into pieces (analysis items into step ranges whose
    covariance partials the solve sums in fp64; at N = 1024 the last 44 utterances'
    synthesis into step pieces with a seam finalize), and a single run splits its one
    utterance the same way, so batch composition moves the fp32 partial sums: every
    utterance must equal its own single-utterance run within the parity tolerance, the same
    batch run twice must agree bitwise, and the peak-normalised output must peak at
    peak / (peak + eps)."""
    from avz import synth
    B, S = 300, 64000
    dm, dt, di = synth.make_batch_device(B, start=77, n_samples=S, n_interferers=2,
                                         device=gpu_device, rng="philox")
    rng = np.random.default_rng(5)
    lens = rng.integers(2000, S + 1, size=B).astype(np.int32)
    lens[:3] = [S, 1024, 16001]
    kw = dict(n_fft=n_fft, sigma=1.0 if mask == "ibm" else 1e-7, mic_d=0.01, mask=mask,
              postfilter="ibm" if mask == "ibm" else "none", normalize="peak", max_samples=S)
    plan = avz.MVDRPlan(max_batch=B, **kw)
    lt = torch.from_numpy(lens).to(gpu_device)
    refs = dict(ref_tgt=dt, ref_int=di) if mask == "ibm" else {}
    out, peak = plan.run(dm, lt, max_len=S, **refs)
    out, peak = out.clone(), peak.clone()
    out2, peak2 = plan.run(dm, lt, max_len=S, **refs)  # run to run: bitwise
    torch.testing.assert_close(out2, out, rtol=0, atol=0, equal_nan=True)
    torch.testing.assert_close(peak2, peak, rtol=0, atol=0, equal_nan=True)
    one = avz.MVDRPlan(max_batch=1, **kw)
    worst = 0.0
    for b in (0, 1, 2, 127, 128, 129, 200, 255, 256, 299):
        L = int(lens[b])
        r1 = (dict(ref_tgt=dt[b:b + 1, :L].contiguous(), ref_int=di[b:b + 1, :L].contiguous())
              if mask == "ibm" else {})
        o1, p1 = one.run(dm[b:b + 1, :, :L].contiguous(), **r1)
        n = one.out_len(L)
        # NaN included: an utterance whose whole output is 0 normalises to 0/0 as the
        # reference's s_out / max|s_out| does (norm_eps 0)
        # batch composition moves the fp32 partial sums' association only
        torch.testing.assert_close(out[b, :n], o1[0, :n], rtol=0, atol=2e-6, equal_nan=True)
        torch.testing.assert_close(peak[b], p1[0], rtol=1e-4, atol=0, equal_nan=True)
        d = (out[b, :n] - o1[0, :n]).abs()
        worst = max(worst, float(d[~d.isnan()].max()) if bool((~d.isnan()).any()) else 0.0)
    print(f"{mask} N={n_fft}: batch vs single runs max |diff| {worst:.2e}")
    n_out = [plan.out_len(int(L)) for L in lens]
    amax = torch.stack([out[b, :n_out[b]].abs().max() for b in range(B)]).double()
    ok = peak > 0  # short utterances inside a silent stretch of the scene beamform to 0
    assert int(ok.sum()) >= 0.95 * B
    assert torch.allclose(amax[ok], torch.ones_like(amax[ok]), rtol=1e-6, atol=0)


@pytest.mark.parametrize("B", [1, 257])
def test_split_batch_unfused_solve_bitwise(avz, gpu_device, B):
    """A split batch with the covariance / weight debug outputs takes the solve kernel and
    the per-utterance kernel's copying instance (pieces included: B = 1 below the CU count,
    B = 257 through the in-kernel piece finalize); its outputs and peaks equal the fused
    in-block solve's -- bitwise at B = 257 (the solve kernel sums each bin's partials in the
    fused solve's order), within 1e-6 at B = 1, whose few bins take the solve lanes kernel
    (fp64 partial sums over 8 lanes combined by a tree: another association) --
    and the debug covariances are finite for every valid bin."""
    from avz import synth
    S = 64000
    dm, dt, di = synth.make_batch_device(B, start=901, n_samples=S, n_interferers=2,
                                         device=gpu_device, rng="philox")
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=B, max_samples=S)
    out, peak = plan.run(dm, ref_tgt=dt, ref_int=di)
    out, peak = out.clone(), peak.clone()
    cov = torch.empty((B, 513, 5), dtype=torch.float64, device=gpu_device)
    w = torch.empty((B, 513, 4), dtype=torch.float32, device=gpu_device)
    out_d, peak_d = plan.run(dm, ref_tgt=dt, ref_int=di, cov_out=cov, w_out=w)
    torch.cuda.synchronize()
    n = plan.out_len(S)
    if B > 1:
        assert torch.equal(out[:, :n], out_d[:, :n])
        assert torch.equal(peak, peak_d)
    else:
        torch.testing.assert_close(out_d[:, :n], out[:, :n], rtol=0, atol=1e-6)
        torch.testing.assert_close(peak_d, peak, rtol=1e-6, atol=0)
    assert bool(torch.isfinite(cov).all())


@pytest.mark.parametrize("B", [257, 300])
def test_piece_finalize_rare_paths_bitwise(avz, gpu_device, B):
    """The in-kernel piece finalize's rare paths, forced through the plan's diagnostics
    (avz_plan_set_diagnostics ipf_mode), give the normal path's output bitwise: (1) every piece but its
    utterance's last arriver hands its interior back at once -- the last arriver rescales the
    pieces that did so before its pass, the others take 1/peak from the pass bit; (2) pieces
    ignore the published 1/peak during their block's next utterance and resolve it at its
    end. The rescale is the same product either way, so outputs and peaks are equal."""
    from avz import synth
    S = 64000
    dm, dt, di = synth.make_batch_device(B, start=77, n_samples=S, n_interferers=2,
                                         device=gpu_device, rng="philox")
    lens = np.full(B, S, np.int32)
    lens[2::5] = np.random.default_rng(B).integers(1024, S + 1, size=len(lens[2::5]))
    lt = torch.from_numpy(lens).to(gpu_device)
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=B, max_samples=S)
    runs = []
    for mode in (0, 1, 2, 0):
        plan.set_diagnostics(synth_variant=2, ipf_mode=mode)
        out, peak = plan.run(dm, lt, max_len=S, ref_tgt=dt, ref_int=di)
        torch.cuda.synchronize()
        runs.append((out.clone(), peak.clone()))
    o0, p0 = runs[0]
    # the valid part of each row (past an utterance's output the row is not written)
    n_out = torch.tensor([plan.out_len(int(L)) for L in lens], device=gpu_device)
    valid = torch.arange(o0.shape[1], device=gpu_device)[None, :] < n_out[:, None]
    for o, p in runs[1:]:
        same = (o == o0) | (torch.isnan(o) & torch.isnan(o0)) | ~valid
        assert bool(same.all()), torch.nonzero(~same)[:8].tolist()
        assert torch.equal(torch.nan_to_num(p, nan=7.0), torch.nan_to_num(p0, nan=7.0))
    ok = torch.from_numpy(lens >= 1024).to(gpu_device)
    amax = torch.where(valid, o0.abs(), torch.zeros_like(o0)).amax(dim=1)[ok]
    fin = torch.isfinite(amax)
    assert torch.allclose(amax[fin], torch.ones_like(amax[fin]), rtol=1e-6, atol=0)


@pytest.mark.parametrize("B", [1, 64, 257, 300])
def test_split_batches_vs_whole_and_oracle(avz, gpu_device, B):
    """Batches that do not fill whole rounds of the persistent grids (configs[1]'s chain at
    B = 1, 64, 257, 300 with ragged lengths): the analysis grid splits its partial last
    round into step-range pieces and the per-utterance synthesis the partial round's (or a
    small batch's) utterances into step pieces with a seam finalize. Utterances on both
    sides of the split (whole, split, the last) against (a) the same utterance run whole
    (a batch of #CU copies: in-block solve, no split), which may differ only by the fp32
    partial sums' association (2e-6), and (b) the oracle (oracle_debug's arithmetic) at the
    parity tolerance, both of them (the IBM decisions are the reference's, frames of the
    generator's silent blocks included: test_gpu_ibm_exact.py). Outputs peak at 1."""
    from avz import synth
    S = 64000
    dm, dt, di = synth.make_batch_device(B, start=4242, n_samples=S, n_interferers=2,
                                         device=gpu_device, rng="philox")
    rng = np.random.default_rng(B)
    lens = np.full(B, S, np.int32)
    if B > 1:
        lens[1::3] = rng.integers(1024, S + 1, size=len(lens[1::3]))
    kw = dict(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm", normalize="peak",
              max_samples=S)
    plan = avz.MVDRPlan(max_batch=B, **kw)
    out, peak = plan.run(dm, torch.from_numpy(lens).to(gpu_device), max_len=S, ref_tgt=dt,
                         ref_int=di)
    torch.cuda.synchronize()
    R = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    whole = avz.MVDRPlan(max_batch=R, **kw)
    # both sides of the split, and up to 8 of the partial round's (piece) utterances
    tail = list(range(B // R * R, B)) if B > R else []
    pick = sorted({0, B // 2, max(B - 2, 0), B - 1} | ({255, 256} & set(range(B))) |
                  set(tail[::max(1, len(tail) // 8)]))
    # every utterance peaks at 1 (a piece interior left unscaled would not)
    ok = lens >= 1024
    n_out = torch.tensor([plan.out_len(int(L)) for L in lens], device=gpu_device)
    valid = torch.arange(out.shape[1], device=gpu_device)[None, :] < n_out[:, None]
    pk = torch.where(valid, out.abs(), torch.zeros_like(out)).amax(dim=1).cpu().numpy()[ok]
    fin = np.isfinite(pk)
    assert np.all(np.abs(pk[fin] - 1.0) <= 1e-6), np.abs(pk[fin] - 1.0).max()
    mix, tgt, itf = (x.cpu().numpy() for x in (dm, dt, di))
    for b in pick:
        L = int(lens[b])
        rep = lambda x: x[b:b + 1, ..., :L].expand(R, *x.shape[1:-1], L).contiguous()  # noqa
        ow, _ = whole.run(rep(dm), ref_tgt=rep(dt), ref_int=rep(di))
        ref = O.oracle_debug_vec(mix[b, :, :L], tgt[b, :L], itf[b, :L], n_fft=1024, hop=512,
                                 sigma=1.0)
        n = len(ref)
        got = out[b, :n].cpu().numpy().astype(np.float64)
        gw = ow[0, :n].cpu().numpy().astype(np.float64)
        if np.isnan(ref).all():  # a silent stretch beamforms to 0: 0 / 0 as the reference's
            assert np.isnan(got).all() and np.isnan(gw).all()
            continue
        d_whole = float(np.max(np.abs(got - gw)))
        e_split, e_whole = float(np.max(np.abs(got - ref))), float(np.max(np.abs(gw - ref)))
        print(f"B={B} b={b} L={L}: |split - whole| {d_whole:.1e}, |split - oracle| "
              f"{e_split:.1e} (at {int(np.argmax(np.abs(got - ref)))}), |whole - oracle| "
              f"{e_whole:.1e}")
        assert d_whole <= 2e-6, (b, L, d_whole)
        assert e_split <= WAVE_TOL and e_whole <= WAVE_TOL, (b, L, e_split, e_whole)
        assert abs(sir(got, tgt[b, :L], itf[b, :L]) - sir(ref, tgt[b, :L], itf[b, :L])) <= SIR_TOL
        assert abs(float(np.max(np.abs(got))) - 1.0) <= 1e-6


def test_piece_seams_ignore_an_earlier_calls_tails(avz, gpu_device):
    """the in-kernel piece finalize forms a split utterance's seams from its
    pieces' halves; the tail slot past its last seam holds no seam of this call (an earlier
    call with another max_len laid its pieces over the slots differently). One plan first runs
    a loud batch of 8-s utterances, then a 4-s batch at B = #CU + 1: the 4-s outputs equal a
    fresh plan's bitwise and peak at 1."""
    from avz import synth
    R = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    B, S1, S2 = R + 1, 128000, 64000
    kw = dict(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
              normalize="peak", max_batch=B, max_samples=S1)
    plan = avz.MVDRPlan(**kw)
    d1 = synth.make_batch_device(B, start=11, n_samples=S1, n_interferers=2,
                                 device=gpu_device, rng="philox")
    plan.run(d1[0] * 1000.0, ref_tgt=d1[1] * 1000.0, ref_int=d1[2] * 1000.0)
    dm, dt, di = synth.make_batch_device(B, start=4242, n_samples=S2, n_interferers=2,
                                         device=gpu_device, rng="philox")
    out, peak = plan.run(dm, ref_tgt=dt, ref_int=di)
    torch.cuda.synchronize()
    fresh = avz.MVDRPlan(**kw)
    out_f, peak_f = fresh.run(dm, ref_tgt=dt, ref_int=di)
    torch.cuda.synchronize()
    n = plan.out_len(S2)
    assert torch.equal(torch.nan_to_num(out[:, :n], nan=7.0), torch.nan_to_num(out_f[:, :n], nan=7.0))
    assert torch.equal(torch.nan_to_num(peak, nan=7.0), torch.nan_to_num(peak_f, nan=7.0))
    amax = out[:, :n].abs().amax(dim=1)
    fin = torch.isfinite(amax)
    assert torch.allclose(amax[fin], torch.ones_like(amax[fin]), rtol=1e-6, atol=0)


def test_piece_interior_resolved_when_later_units_are_skipped(avz, gpu_device):
    """a piece's interior rescale waits lazily for its utterance's 1/peak
    and is resolved at the end of its block's next whole utterance -- or, when the block has
    none left to run (device lengths below N: skipped), right after its loop. B = #CU + 1 with
    the first #CU rows of device length 0: the split last utterance equals its single run
    (within the fp32 association, 2e-6) and peaks at 1."""
    from avz import synth
    R = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    B, S = R + 1, 64000
    dm, dt, di = synth.make_batch_device(B, start=4242, n_samples=S, n_interferers=2,
                                         device=gpu_device, rng="philox")
    lens = torch.zeros(B, dtype=torch.int32, device=gpu_device)
    lens[B - 1] = S
    kw = dict(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
              normalize="peak", max_samples=S)
    plan = avz.MVDRPlan(max_batch=B, **kw)
    out, peak = plan.run(dm, lens, max_len=S, ref_tgt=dt, ref_int=di)
    one = avz.MVDRPlan(max_batch=1, **kw)
    o1, p1 = one.run(dm[B - 1:].contiguous(), ref_tgt=dt[B - 1:].contiguous(),
                     ref_int=di[B - 1:].contiguous())
    torch.cuda.synchronize()
    n = plan.out_len(S)
    d = float((out[B - 1, :n] - o1[0, :n]).abs().max())
    assert d <= 2e-6, d
    assert abs(float(out[B - 1, :n].abs().max()) - 1.0) <= 1e-6
