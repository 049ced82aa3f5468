"""Size-independent properties of the HIP chain at the bench configuration (B = 256
utterances of 4.0 s, 1024/512, oracle IBM, BASELINE configs[1]) and edge sizes:
run-to-run determinism, batch-order invariance, scale invariance of the peak-normalised
output at sigma = 0, the oracle on sampled utterances of the full batch, and the
extreme lengths a plan accepts."""
import numpy as np
import pytest
import torch

from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu

B, S, N = 256, 64000, 1024


@pytest.fixture(scope="module")
def full_batch(gpu_device):
    import avz
    from avz import synth
    mix, tgt, itf = synth.make_batch(B, start=0, n_samples=S, n_interferers=2)
    d = lambda a: torch.from_numpy(a).to(gpu_device)  # noqa: E731
    return avz, mix, tgt, itf, d(mix), d(tgt), d(itf)


def _plan(avz, sigma=1.0, max_batch=B, max_samples=S):
    return avz.MVDRPlan(n_fft=N, sigma=sigma, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=max_batch, max_samples=max_samples)


def test_deterministic_and_order_invariant(full_batch):
    avz, mix, tgt, itf, dm, dt, di = full_batch
    plan = _plan(avz)
    o1, p1 = plan.run(dm, ref_tgt=dt, ref_int=di)
    o1 = o1.clone()
    o2, _ = plan.run(dm, ref_tgt=dt, ref_int=di)
    assert torch.equal(o1, o2)  # no float atomics on the data path: bitwise repeatable
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(0)).to(dm.device)
    o3, p3 = plan.run(dm[perm].contiguous(), ref_tgt=dt[perm].contiguous(),
                      ref_int=di[perm].contiguous())
    assert torch.equal(o3, o1[perm]) and torch.equal(p3, p1[perm])


def test_full_batch_matches_oracle_on_samples(full_batch):
    avz, mix, tgt, itf, dm, dt, di = full_batch
    out, peak = _plan(avz).run(dm, ref_tgt=dt, ref_int=di)
    n_out = O.n_frames(S, N, N // 2) * (N // 2) - N // 2
    for b in (0, 77, 255):
        ref = O.oracle_debug_vec(mix[b], tgt[b], itf[b], n_fft=N, hop=N // 2, sigma=1.0)
        got = out[b, :n_out].cpu().numpy().astype(np.float64)
        assert np.max(np.abs(got - ref)) <= 1e-4
        L = S
        d_sir = abs(O.projection_sdr_sir(got[:L], tgt[b], itf[b])[1]
                    - O.projection_sdr_sir(ref[:L], tgt[b], itf[b])[1])
        assert d_sir <= 0.01


def test_scale_invariance_sigma0(full_batch):
    """At sigma = 0 the MVDR weights are invariant to the mixture's scale and the output
    is peak-normalised, so chain(2^k mix) == chain(mix) up to the +1e-10 in the
    distortionless normalisation (exact power-of-two scaling in fp32)."""
    avz, mix, tgt, itf, dm, dt, di = full_batch
    k = 32
    plan = _plan(avz, sigma=0.0, max_batch=k)
    o1, p1 = plan.run(dm[:k].contiguous(), ref_tgt=dt[:k].contiguous(), ref_int=di[:k].contiguous())
    o1 = o1.clone()
    o2, p2 = plan.run((dm[:k] * 4.0).contiguous(), ref_tgt=dt[:k].contiguous(),
                      ref_int=di[:k].contiguous())
    assert torch.max(torch.abs(o1 - o2)).item() <= 1e-5
    torch.testing.assert_close(p2, 4.0 * p1, rtol=1e-5, atol=0)


@pytest.mark.parametrize("length", [N, N + 1, S])
def test_edge_lengths(gpu_device, length):
    """The shortest utterance a plan accepts (n_fft; scipy needs nperseg <= L), one past
    it, and the plan maximum, in one ragged launch with a zero-length-padded neighbour."""
    import avz
    rng = np.random.default_rng(length)
    lens = [length, S]
    x = np.zeros((2, 2, S), np.float32)
    t = np.zeros((2, S), np.float32)
    i = np.zeros((2, S), np.float32)
    for b, L in enumerate(lens):
        x[b, :, :L] = 0.1 * rng.standard_normal((2, L))
        t[b, :L] = 0.1 * rng.standard_normal(L)
        i[b, :L] = 0.1 * rng.standard_normal(L)
    plan = _plan(avz, max_batch=2)
    d = lambda a: torch.from_numpy(a).to(gpu_device)  # noqa: E731
    ln = torch.tensor(lens, dtype=torch.int32, device=gpu_device)
    out, _ = plan.run(d(x), ln, max_len=S, ref_tgt=d(t), ref_int=d(i))
    for b, L in enumerate(lens):
        ref = O.oracle_debug_vec(x[b, :, :L], t[b, :L], i[b, :L], n_fft=N, hop=N // 2, sigma=1.0)
        got = out[b, :len(ref)].cpu().numpy().astype(np.float64)
        assert np.max(np.abs(got - ref)) <= 1e-4
    # lengths outside the plan are rejected, never run
    with pytest.raises(avz.AvzError):
        plan.run(d(x[:, :, :N - 1].copy()), ref_tgt=d(t[:, :N - 1].copy()),
                 ref_int=d(i[:, :N - 1].copy()))
