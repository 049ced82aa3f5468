"""On-device scene generator (avz_scene_mix) against the host generator
avz/synth.make_scene, whose fractional delay restates world_building.py:53-59 (pinned by
tests/test_scene_formats.py). The device path runs the delay as an fp32 circular
convolution with the exact periodic kernel, so the tolerance is fp32 accumulation over
S terms: 2e-5 absolute on the peak-normalised outputs."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,k,batch", [(16000, 2, 6), (64000, 3, 2), (8000, 0, 3)])
def test_device_scene_matches_host(gpu_device, n, k, batch):
    from avz import synth
    mix, tgt, itf = synth.make_batch_device(batch, start=5, n_samples=n, n_interferers=k,
                                            device=gpu_device)
    hm, ht, hi = synth.make_batch(batch, start=5, n_samples=n, n_interferers=k)
    for a, h in ((mix, hm), (tgt, ht), (itf, hi)):
        assert np.max(np.abs(a.cpu().numpy() - h)) <= 2e-5
    assert abs(float(mix.abs().amax()) - 1.0) <= 1e-6 or k == 0


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
    print(f"device scene generation, {B} x 4 s: {dt * 1e3:.1f} ms (incl. host draws)")
