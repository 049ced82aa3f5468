"""Full-size parity of BASELINE configs[3] and configs[4] on the HIP path: ONE launch over
the whole single-GPU workload, the oracle on sampled utterances / items.

configs[3]: B = 1024 utterances of 4.0 s (2 interferers, avz_scene_generate on the device,
as bench.py generates them), heuristic IPD mask (rt_av_zoom/core/masked_mvdr.py:37-46),
1024/512, sigma 1e-7, peak normalisation + 1e-6 — one MVDRPlan.run; on sampled utterances
the oracle's masked_mvdr_vec: 0 differing IPD mask decisions (per-bin mask-weight sums,
cov_out column 4), waveform max-abs <= 1e-4, SIR |d| <= 0.01 dB.

configs[4]'s MVDR chain: the same 1024 utterances cut into 4096 two-second items
(avz_chunk_split, full_audio_generating_pipeline/inference.py:120-167's windows) through the
external-mask chain (sigma 1e-5, d 0.04, max(M, 0.05) post-filter, 100 Hz skip) with a
seeded random target mask — one MVDRPlan.run; sampled items against
O.external_mask_vec (waveform max-abs <= 1e-4 of the item's peak).

Whole-batch properties (size-independent): run-to-run bitwise determinism, the debug
outputs (cov_out) not changing the product output, finite everywhere, every peak-normalised
utterance's max |out| = peak / (peak + 1e-6)."""
import numpy as np
import pytest
import torch

from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu

B, S, K, N = 1024, 64000, 2, 1024
SAMPLE_UTTS = (0, 1, 257, 511, 512, 777, 1022, 1023)
SAMPLE_ITEMS = (0, 1, 2, 3, 1029, 2047, 2048, 3333, 4094, 4095)


@pytest.fixture(scope="module")
def batch(gpu_device):
    from avz import synth
    return synth.make_batch_device(B, start=0, n_samples=S, n_interferers=K, device=gpu_device,
                                   rng="philox")


def test_configs3_ipd_full_batch(gpu_device, batch):
    import avz
    dm, dt, di = batch
    plan = avz.MVDRPlan(n_fft=N, sigma=1e-7, mic_d=0.01, mask="ipd", postfilter="none",
                        normalize="peak", norm_eps=1e-6, max_batch=B, max_samples=S)
    F = N // 2 + 1
    out, peak = plan.run(dm)
    out, peak = out.clone(), peak.clone()
    cov = torch.zeros((B, F, 5), dtype=torch.float64, device=gpu_device)
    out2, peak2 = plan.run(dm, cov_out=cov)
    assert torch.equal(out, out2) and torch.equal(peak, peak2)
    n_out = plan.out_len(S)
    o = out[:, :n_out]
    assert torch.isfinite(o).all() and torch.isfinite(cov).all()
    amax = o.abs().amax(dim=1).double()
    pk = peak.double()
    assert torch.allclose(amax, pk / (pk + 1e-6), rtol=1e-6, atol=0)
    msum_all = cov[:, :, 4].cpu().numpy()
    worst_w, worst_sir, n_dec, n_bins = 0.0, 0.0, 0, 0
    for b in SAMPLE_UTTS:
        mix, tgt, itf = dm[b].cpu().numpy(), dt[b].cpu().numpy(), di[b].cpu().numpy()
        ref, st = O.masked_mvdr_vec(mix, n_fft=N, hop=N // 2, return_stages=True)
        rsum = st["mask"].astype(np.float64).sum(axis=1)
        n_dec += int(np.sum(np.round(np.abs(msum_all[b] - rsum) / 0.99)))
        n_bins += st["mask"].size
        got = o[b].cpu().numpy().astype(np.float64)
        assert len(got) == len(ref)
        worst_w = max(worst_w, float(np.max(np.abs(got - ref))))
        d_sir = abs(O.projection_sdr_sir(got[:S], tgt, itf)[1]
                    - O.projection_sdr_sir(ref[:S], tgt, itf)[1])
        worst_sir = max(worst_sir, d_sir)
    print(f"configs[3] B={B}: {len(SAMPLE_UTTS)} sampled utterances, IPD decisions differing "
          f"{n_dec} of {n_bins}, worst waveform |d| {worst_w:.2e}, worst SIR |d| "
          f"{worst_sir:.2e} dB")
    assert n_dec == 0
    assert worst_w <= 1e-4 and worst_sir <= 0.01
    out3, _ = plan.run(dm)
    assert torch.equal(out3, out)


def test_configs4_external_chain_4096_items(gpu_device, batch):
    from avz import neural as NM
    dm = batch[0]
    bf = NM.NeuralMaskBeamformer(torch.nn.Identity(), max_items=4 * B)
    items = bf.split(dm)[0]
    n = items.shape[0]
    assert n == 4 * B
    F, T = bf.plan.cfg.n_fft // 2 + 1, bf.plan.frames(bf.chunk)
    g = torch.Generator(device=gpu_device).manual_seed(7)
    mask = torch.rand((n, F, T), generator=g, device=gpu_device)
    out, peak = bf.plan.run(items, ext_mask=mask)
    out, peak = out.clone(), peak.clone()
    n_out = bf.plan.out_len(bf.chunk)
    assert torch.isfinite(out[:, :n_out]).all()
    assert torch.equal(peak, out[:, :n_out].abs().amax(dim=1))
    out2, _ = bf.plan.run(items, ext_mask=mask)
    assert torch.equal(out2, out)
    worst = 0.0
    for i in SAMPLE_ITEMS:
        x = items[i].cpu().numpy()
        M = mask[i].cpu().numpy()
        ref = O.external_mask_vec(x, M, n_fft=1024, hop=512, sigma=1e-5, d=0.04, floor=0.05)
        got = out[i, :len(ref)].cpu().numpy().astype(np.float64)
        assert len(ref) == n_out
        scale = np.max(np.abs(ref))
        worst = max(worst, float(np.max(np.abs(got - ref)) / scale))
    print(f"configs[4] chain: {n} items, {len(SAMPLE_ITEMS)} sampled, worst |d| / peak "
          f"{worst:.2e}")
    assert worst <= 1e-4
