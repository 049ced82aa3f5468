"""GPU parity of the neural-mask path (BASELINE configs[4]; full_audio_generating_pipeline/
inference.py process_chunk + main_deploy): device features -> U-Net (PyTorch-ROCm) ->
HIP MVDR chain (external mask, max(M, 0.05) post-filter) -> chunk overlap-add, against
the reference run with the same seeded U-Net weights (tests/golden/neural_*.npz).

Tolerances: with the reference's own masks fed in (the HIP chain alone) waveform max-abs
<= 1e-4 and SIR |delta| <= 0.01 dB; end to end with the U-Net on the GPU (MIOpen fp32
convolutions vs the reference's CPU convolutions: masks agree to ~1e-5) the same bars."""
import os

import numpy as np
import pytest
import torch

from conftest import golden, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu

WAVE_TOL = 1e-4
SIR_TOL = 0.01


@pytest.fixture(scope="module")
def neural(gpu_device):
    from avz import neural as N
    g = golden("neural_excerpt_test.npz")
    torch.manual_seed(int(g["seed"]))
    model = N.FreqPreservingUNet().eval().to(gpu_device)
    return N, model


def sir(out, tgt, itf):
    L = min(len(out), len(tgt))
    return O.projection_sdr_sir(out[:L].astype(np.float64), tgt[:L], itf[:L])[1]


def test_hip_chain_with_reference_masks(neural, gpu_device):
    N, model = neural
    g = golden("neural_excerpt_test.npz")
    mix, tgt, itf = triple_f32("test", g["seg"])
    bf = N.NeuralMaskBeamformer(model, max_items=len(g["masks"]))
    masks = torch.from_numpy(g["masks"]).to(gpu_device)
    y, _ = bf.run(torch.from_numpy(mix)[None].to(gpu_device), mask_fn=lambda items: masks)
    out = y[0].cpu().numpy().astype(np.float64)
    ref = g["out"].astype(np.float64)
    assert out.shape == ref.shape
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - sir(ref, tgt, itf)) <= SIR_TOL


def test_device_unet_masks(neural, gpu_device):
    """The U-Net on the device from the reference's own chunk-0 features: MIOpen fp32
    vs the reference's CPU convolutions. (The device features themselves are checked
    against the reference's in test_gpu_features.py; a bin whose IPD sits on the +-pi
    cut may take the other branch there, which moves the mask locally by up to ~5e-3 —
    the end-to-end tests below bound what that does to the output.)"""
    N, model = neural
    g = golden("neural_excerpt_test.npz")
    with torch.no_grad():
        m = model(torch.from_numpy(g["feat0"])[None].to(gpu_device))[0].cpu().numpy()
    assert np.max(np.abs(m - g["masks"][0])) <= 1e-4


@pytest.mark.parametrize("trip", ["test", "set2"])
def test_end_to_end_vs_reference(neural, gpu_device, trip):
    N, model = neural
    g = golden(f"neural_{trip}.npz")
    mix, tgt, itf = triple_f32(trip)
    S = mix.shape[1]
    bf = N.NeuralMaskBeamformer(model, max_items=-(-S // 16000))
    y, _ = bf.run(torch.from_numpy(mix)[None].to(gpu_device))
    out = y[0].cpu().numpy().astype(np.float64)
    assert len(out) == int(g["out_len"])
    assert np.max(np.abs(out[::16] - g["out_stride16"])) <= WAVE_TOL
    assert np.max(np.abs(out[:4096] - g["out_head"])) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - float(g["sir_out"])) <= SIR_TOL


def test_ragged_batch_equals_single(neural, gpu_device):
    """One chain launch over all chunks of a ragged batch == utterance by utterance."""
    N, model = neural
    mix, _, _ = triple_f32("test")
    lens = [48000, 31000, 64000, 16001]
    S = max(lens)
    x = np.zeros((len(lens), 2, S), np.float32)
    for b, L in enumerate(lens):
        x[b, :, :L] = mix[:, 1000 * b:1000 * b + L]
    bf = N.NeuralMaskBeamformer(model, max_items=sum(-(-L // 16000) for L in lens))
    y, _ = bf.run(torch.from_numpy(x).to(gpu_device), lengths=lens)
    for b, L in enumerate(lens):
        bf1 = N.NeuralMaskBeamformer(model, max_items=-(-L // 16000))
        y1, _ = bf1.run(torch.from_numpy(np.ascontiguousarray(x[b:b + 1, :, :L])).to(gpu_device))
        got = y[b, :L].cpu().numpy()
        exp = y1[0].cpu().numpy()
        # the HIP chain is per-item identical; MIOpen may pick another convolution
        # algorithm for another batch size, so the masks may differ in the last bits
        assert np.max(np.abs(got - exp)) <= 1e-5
        assert np.all(y[b, L:].cpu().numpy() == 0)


def test_main_deploy_file_mirror(neural, gpu_device, tmp_path, monkeypatch):
    N, model = neural
    from avz import wavio
    mix, _, _ = triple_f32("test", (40000, 88000))
    wavio.write(str(tmp_path / "input.wav"), mix.T, 16000)
    monkeypatch.chdir(tmp_path)
    out = N.main_deploy(str(tmp_path / "input.wav"), model=model)
    assert os.path.exists(tmp_path / "enhanced_input.wav")
    ref = golden("neural_excerpt_test.npz")["out"]
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    assert N.main_deploy(str(tmp_path / "input.wav"), model_path=str(tmp_path / "absent.pth")) is None


def test_refresh_after_weight_change(neural, gpu_device):
    """fold_bn snapshots the caller's weights (a BatchNorm-folded copy): a later change to
    the caller's model is not seen until refresh(model) rebuilds the copy."""
    import copy
    N, model0 = neural
    model = copy.deepcopy(model0)
    bf = N.NeuralMaskBeamformer(model, max_items=2)
    x = torch.randn((2, 2, 16000), device=gpu_device)
    items = bf.split(x)[0]
    m0 = bf.masks(items).clone()
    with torch.no_grad():
        for p in model.parameters():
            p.mul_(1.5)
    torch.testing.assert_close(bf.masks(items), m0, rtol=0, atol=0)  # the snapshot
    bf.refresh(model)
    m1 = bf.masks(items)
    with torch.no_grad():
        ref = model(N.mask_features(bf.plan, items, "unet"))
    assert not torch.equal(m1, m0)
    torch.testing.assert_close(m1, ref, rtol=1e-4, atol=1e-5)
