"""GPU parity of the Final_pipeline path: hybrid hard-null beamformer (AVZ_BF_HYBRID_NULL)
inside the chunked driver (avz_chunk_split -> avz_mvdr_batch -> avz_chunk_merge), against
the reference's own enhance_audio output (tests/golden/hybrid_*.npz) and the oracle.
Tolerances as the core path: peak-normalised waveform max-abs <= 1e-4, SIR |d| <= 0.01 dB."""
import os

import numpy as np
import pytest
import torch

from conftest import golden, hybrid_bin_causes, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu

WAVE_TOL = 1e-4
SIR_TOL = 0.01


@pytest.fixture(scope="module")
def fp(gpu_device):
    from avz import final_pipeline
    return final_pipeline


def dev_t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("trip", ["test", "set2"])
def test_chunked_hybrid_matches_reference(fp, gpu_device, trip):
    g = golden(f"hybrid_{trip}.npz")
    mix, t, i = triple_f32(trip)
    S = mix.shape[1]
    bf = fp.ChunkedHybridBeamformer(max_items=-(-S // 16000), mask="ibm")
    y, peak = bf.run(dev_t(mix, gpu_device)[None], ref_tgt=dev_t(t[:S], gpu_device)[None],
                     ref_int=dev_t(i[:S], gpu_device)[None])
    out = y[0].cpu().numpy().astype(np.float64)
    assert out.shape == g["out"].shape
    err = np.abs(out - g["out"]).max()
    assert err <= WAVE_TOL, err
    L = min(len(out), len(t))
    sir = O.projection_sdr_sir(out[:L], t[:L], i[:L])[1]
    assert abs(sir - g["sir_out"]) <= SIR_TOL
    assert float(peak[0]) > 0


def test_hybrid_weights_vs_oracle(fp, gpu_device):
    """Per-bin weights of chunk 0 (w_out debug output) against the closed-form restatement
    on the reference's own chunk-0 STFT and mask."""
    import avz
    g = golden("hybrid_test.npz")
    mix, t, i = triple_f32("test")
    plan = avz.MVDRPlan(n_fft=1024, mic_d=0.08, mask="ibm", postfilter="ibm",
                        beamformer="hybrid_null", normalize="none", max_batch=1,
                        max_samples=32000)
    w = torch.zeros((1, 513, 4), dtype=torch.float32, device=gpu_device)
    cov = torch.zeros((1, 513, 5), dtype=torch.float64, device=gpu_device)
    plan.run(dev_t(mix[:, :32000], gpu_device)[None], ref_tgt=dev_t(t[:32000], gpu_device)[None],
             ref_int=dev_t(i[:32000], gpu_device)[None], w_out=w, cov_out=cov)
    wg = w[0].cpu().numpy().astype(np.float64)
    Wg = np.stack([wg[:, 0] + 1j * wg[:, 1], wg[:, 2] + 1j * wg[:, 3]], axis=1)
    Y, M, f = g["chunk0_Y"], g["chunk0_mask"], g["chunk0_f"]
    Wo = O.hybrid_weights_vec(Y, M, f)
    close = np.abs(Wg - Wo).max(axis=1) <= 1e-3 * np.maximum(1.0, np.abs(Wo).max(axis=1))
    assert (np.abs(Wg[:13] - [1, 0]) == 0).all()
    # every bin whose weights differ must be explained (conftest.hybrid_bin_causes)
    cnt_gpu = cov[0, :, 4].cpu().numpy()
    causes = hybrid_bin_causes(
        Y, M, f, np.nonzero(~close)[0],
        lambda k, w: np.abs(Wg[k] - w).max() <= 1e-3 * max(1.0, np.abs(w).max()), cnt=cnt_gpu)
    print(f"hybrid chunk 0: {int((~close).sum())} of {len(close)} bins differ: {causes}")


def test_external_mask_equals_ibm_mode(fp, gpu_device):
    """The same oracle target mask fed as an external mask (x M post-filter, noise 1 - M)
    reproduces the IBM mode."""
    mix, t, i = triple_f32("test", seg=(0, 48000))
    S = mix.shape[1]
    d = gpu_device
    ibm = fp.ChunkedHybridBeamformer(max_items=3, mask="ibm")
    y0, _ = ibm.run(dev_t(mix, d)[None], ref_tgt=dev_t(t, d)[None], ref_int=dev_t(i, d)[None])
    ext = fp.ChunkedHybridBeamformer(max_items=3, mask="external")
    masks = np.stack([O.chunk_target_mask(t, i, s) for s in range(0, S, 16000)])

    def mask_fn(items):
        assert items.shape == (3, 2, 32000)
        return dev_t(masks, d)
    y1, _ = ext.run(dev_t(mix, d)[None], mask_fn=mask_fn)
    assert torch.allclose(y0, y1, atol=2e-5)


def test_ragged_batch_equals_single(fp, gpu_device):
    d = gpu_device
    mix, t, i = triple_f32("set2")
    lens = [40000, 110000, 16000]
    S = max(lens)
    B = len(lens)
    M = np.zeros((B, 2, S), np.float32)
    T = np.zeros((B, S), np.float32)
    I = np.zeros((B, S), np.float32)
    for b, L in enumerate(lens):
        off = 3000 * b
        M[b, :, :L] = mix[:, off:off + L]
        T[b, :L] = t[off:off + L]
        I[b, :L] = i[off:off + L]
    bf = fp.ChunkedHybridBeamformer(max_items=sum(-(-L // 16000) for L in lens), mask="ibm")
    y, _ = bf.run(dev_t(M, d), lengths=lens, ref_tgt=dev_t(T, d), ref_int=dev_t(I, d))
    for b, L in enumerate(lens):
        one = fp.ChunkedHybridBeamformer(max_items=-(-L // 16000), mask="ibm")
        y1, _ = one.run(dev_t(M[b:b + 1, :, :L], d), ref_tgt=dev_t(T[b:b + 1, :L], d),
                        ref_int=dev_t(I[b:b + 1, :L], d))
        assert torch.equal(y[b, :L], y1[0])
        assert (y[b, L:] == 0).all()


def test_enhance_audio_mirror(fp, gpu_device, tmp_path):
    from avz import wavio
    g = golden("hybrid_test.npz")
    mix, t, i = triple_f32("test")
    run = tmp_path / "sim" / "run1"
    run.mkdir(parents=True)
    wavio.write(str(run / "mixture.wav"), mix.T, 16000)
    wavio.write(str(run / "target.wav"), np.stack([t, t], 1), 16000)
    wavio.write(str(run / "interference.wav"), np.stack([i, i], 1), 16000)
    out = fp.enhance_audio("run1", str(run / "mixture.wav"), "absent.tflite",
                           results_dir=str(tmp_path / "results"))
    path = tmp_path / "results" / "run1_results" / "run1_enhanced.wav"
    assert os.path.exists(path)
    back, fs = wavio.read(str(path))
    assert fs == 16000 and back.shape == g["out"].shape
    assert np.abs(out - g["out"]).max() <= WAVE_TOL
    assert np.abs(back - g["out"]).max() <= 1.0 / 32768 + WAVE_TOL
