"""Neural-mask path (full_audio_generating_pipeline/inference.py) on the CPU: the U-Net
mirror's state_dict layout and seeded init against the reference's own model, its
forward against the reference's recorded mask, and the CPU restatement of
process_chunk/main_deploy against the reference run (tests/golden/neural_*.npz)."""
import numpy as np
import pytest
import torch

from conftest import golden, triple_f32
from oracle import avz_oracle as O


def checksum(state_dict):
    n, s1, s2 = 0, 0.0, 0.0
    for k in sorted(state_dict):
        v = state_dict[k].detach().double().flatten().numpy()
        n += v.size
        s1 += float(np.abs(v).sum())
        s2 += float((v * np.linspace(1.0, 2.0, v.size)).sum())
    return np.array([n, s1, s2])


@pytest.fixture(scope="module")
def unet():
    from avz.neural import FreqPreservingUNet
    g = golden("neural_excerpt_test.npz")
    torch.manual_seed(int(g["seed"]))
    return FreqPreservingUNet().eval(), g


def test_unet_state_dict_matches_reference(unet):
    model, g = unet
    sd = model.state_dict()
    assert sorted(sd) == list(g["keys"])
    np.testing.assert_allclose(checksum(sd), g["checksum"], rtol=1e-12)


def test_unet_forward_matches_reference_mask(unet):
    model, g = unet
    with torch.no_grad():
        m = model(torch.from_numpy(g["feat0"])[None]).numpy()[0]
    np.testing.assert_allclose(m, g["masks"][0], atol=1e-6)


def test_batchnorm_folded_unet_matches_reference_mask(unet):
    """fold_batchnorm (the inference copy NeuralMaskBeamformer runs): no BatchNorm left,
    the original model untouched, and the same reference mask within fp32 rounding —
    with the reference's fresh BN statistics and with non-trivial ones."""
    from avz.neural import fold_batchnorm
    model, g = unet
    folded = fold_batchnorm(model)
    assert not any(isinstance(m, torch.nn.BatchNorm2d) for m in folded.modules())
    assert any(isinstance(m, torch.nn.BatchNorm2d) for m in model.modules())
    x = torch.from_numpy(g["feat0"])[None]
    with torch.no_grad():
        np.testing.assert_allclose(folded(x).numpy()[0], g["masks"][0], atol=1e-6)
    import copy
    m2 = copy.deepcopy(model)
    gen = torch.Generator().manual_seed(3)
    for bn in (m for m in m2.modules() if isinstance(m, torch.nn.BatchNorm2d)):
        bn.running_mean.copy_(torch.rand(bn.num_features, generator=gen) - 0.5)
        bn.running_var.copy_(torch.rand(bn.num_features, generator=gen) + 0.5)
        bn.weight.data.copy_(torch.rand(bn.num_features, generator=gen) + 0.5)
        bn.bias.data.copy_(torch.rand(bn.num_features, generator=gen) - 0.5)
    with torch.no_grad():
        a, b = m2(x), fold_batchnorm(m2)(x)
    assert float((a - b).abs().max()) <= 1e-6
    with pytest.raises(ValueError):
        fold_batchnorm(copy.deepcopy(model).train())


def test_unet_features_oracle(unet):
    _, g = unet
    mix, _, _ = triple_f32("test", g["seg"])
    feat = O.mask_features(mix[:, :32000], n_fft=1024, layout="unet")
    ref = g["feat0"]
    np.testing.assert_allclose(feat[0], ref[0], atol=1e-5)
    # IPD: equal up to the 2 pi branch of angle() differences computed at the cut
    d = np.abs(feat[1] - ref[1])
    assert np.all((d < 1e-5) | (np.abs(d - 2 * np.pi) < 1e-4))


def test_neural_deploy_oracle_vs_reference():
    g = golden("neural_excerpt_test.npz")
    mix, _, _ = triple_f32("test", g["seg"])
    out = O.neural_deploy_vec(mix.T, g["masks"], chunk=int(g["chunk"]), n_fft=int(g["n_fft"]),
                              d=float(g["mic_d"]), sigma=float(g["sigma"]))
    np.testing.assert_allclose(out, g["out"], atol=2e-6)
