"""On-device scene generator.

* avz_scene_mix (host draws) against the host generator avz/synth.make_scene, whose
  fractional delay restates world_building.py:53-59 (pinned by tests/test_scene_formats.py).
  The delays run as fp64 mixed-radix FFTs (lengths 2^a 3^b 5^c) or, for other lengths, as
  the exact O(n^2) fp32 circular convolution; tolerance 2e-5 absolute on the
  peak-normalised outputs (fp32 accumulation over n terms on the fallback).
* avz_scene_generate (everything on the device, counter-based draws) against its host
  restatement synth.make_batch_philox, and the generation time of a configs[2] shard
  (512 utterances x 4 s, 3 interferers)."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,k,batch", [(16000, 2, 6), (64000, 3, 2), (8000, 0, 3),
                                       (14000, 2, 2)])
def test_device_scene_matches_host(gpu_device, n, k, batch):
    from avz import synth
    mix, tgt, itf = synth.make_batch_device(batch, start=5, n_samples=n, n_interferers=k,
                                            device=gpu_device)
    hm, ht, hi = synth.make_batch(batch, start=5, n_samples=n, n_interferers=k)
    worst = max(float(np.max(np.abs(a.cpu().numpy() - h))) for a, h in ((mix, hm), (tgt, ht),
                                                                         (itf, hi)))
    path = "fft" if n != 14000 else "O(n^2) convolution"
    print(f"avz_scene_mix n={n} k={k} ({path}): max |d| {worst:.2e}")
    assert worst <= 2e-5
    assert abs(float(mix.abs().amax()) - 1.0) <= 1e-6 or k == 0


@pytest.mark.parametrize("n,k,batch,start", [(64000, 3, 3, 0), (16000, 2, 4, 1000),
                                             (8000, 0, 2, 7), (64000, 1, 2, 2 ** 33 + 5)])
def test_generated_scene_matches_restatement(gpu_device, n, k, batch, start):
    from avz import synth
    mix, tgt, itf = synth.make_batch_device(batch, start=start, n_samples=n, n_interferers=k,
                                            device=gpu_device, rng="philox")
    hm, ht, hi = synth.make_batch_philox(batch, start=start, n_samples=n, n_interferers=k)
    worst = max(float(np.max(np.abs(a.cpu().numpy() - h))) for a, h in ((mix, hm), (tgt, ht),
                                                                         (itf, hi)))
    print(f"avz_scene_generate n={n} k={k} start={start}: max |d| vs host restatement {worst:.2e}")
    assert worst <= 2e-5
    assert abs(float(mix.abs().amax()) - 1.0) <= 1e-6 or k == 0
    # another seed is another scene
    m2, _, _ = synth.make_batch_device(batch, start=start, n_samples=n, n_interferers=k,
                                       device=gpu_device, rng="philox", seed=1)
    assert not torch.equal(mix, m2)


def test_configs2_shard_generation_time(gpu_device):
    """A configs[2] per-GPU shard (512 x 4 s, 3 interferers) is generated on the device in
    well under the 50 ms target; sampled utterances equal the host restatement."""
    from avz import synth
    B, S, K = 512, 64000, 3
    synth.make_batch_device(8, n_samples=S, n_interferers=K, device=gpu_device, rng="philox")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mix, tgt, itf = synth.make_batch_device(B, n_samples=S, n_interferers=K, device=gpu_device,
                                            rng="philox")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"configs[2] shard generated on the device: {dt * 1e3:.1f} ms ({B} x {S} x {K + 1} src)")
    assert dt < 0.05
    for b in (0, 311):
        hm, ht, hi = synth.make_scene_philox(b, S, K)
        assert np.max(np.abs(mix[b].cpu().numpy() - hm)) <= 2e-5
        assert np.max(np.abs(tgt[b].cpu().numpy() - ht)) <= 2e-5


def test_device_scene_feeds_the_chain(gpu_device):
    """A device-generated batch through the IBM chain gives the SIR the host batch gives."""
    import avz
    from avz import metrics, synth
    B, S = 16, 64000
    t0 = time.perf_counter()
    mix, tgt, itf = synth.make_batch_device(B, start=100, n_samples=S, device=gpu_device)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=B, max_samples=S)
    out, _ = plan.run(mix, ref_tgt=tgt, ref_int=itf)
    hm, ht, hi = synth.make_batch(B, start=100, n_samples=S)
    d = lambda a: torch.from_numpy(a).to(gpu_device)  # noqa: E731
    out_h, _ = plan.run(d(hm), ref_tgt=d(ht), ref_int=d(hi))
    sir_d = metrics.projection_metrics(out[:, :S], tgt, itf)[:, 3]
    sir_h = metrics.projection_metrics(out_h[:, :S], d(ht), d(hi))[:, 3]
    assert torch.max(torch.abs(sir_d - sir_h)).item() <= 1e-3
    print(f"device scene mixing, {B} x 4 s: {dt * 1e3:.1f} ms (incl. host draws)")
