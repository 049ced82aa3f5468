"""tf_lite_version's process_audio_file (rt_av_zoom/core/tf_lite_version/inference.py:245-391)
against the reference run itself on the bundled mixtures (tests/golden/tflite_*.npz, make_golden.py gen_tflite):
the absent TFLite model is replaced by a mask feeder handing each chunk a fixed soft target
mask (stored in the fixture), so the reference's output is reproducible.

CPU: the oracle restatement (O.process_audio_file_vec) is pinned to the fixtures.
GPU: the engine mirror (avz.tflite_pipeline.process_audio_file, file in -> file out) with
mask_fn returning the same masks; peak-normalised waveform max-abs <= 1e-4, SIR |d| <= 0.01
dB, and the chunk-0 model features it hands mask_fn against the ones the reference handed
its model (fp32 STFT vs scipy's fp64: tolerance as tests/test_gpu_features.py)."""
import numpy as np
import pytest

from conftest import golden, triple_f32
from oracle import avz_oracle as O

TRIPS = ["test", "set2"]
WAVE_TOL = 1e-4
SIR_TOL = 0.01


@pytest.mark.parametrize("trip", TRIPS)
def test_oracle_matches_reference_run(trip):
    g = golden(f"tflite_{trip}.npz")
    mix, t, i = triple_f32(trip)
    out = O.process_audio_file_vec(mix.T, g["masks"], chunk=int(g["chunk"]),
                                   n_fft=int(g["n_fft"]), d=float(g["d"]), c=float(g["c"]),
                                   sigma=float(g["sigma"]))
    assert len(out) == int(g["out_len"]) == mix.shape[1]
    np.testing.assert_allclose(out, g["out"], atol=5e-7)
    L = min(len(out), len(t))
    sir = O.projection_sdr_sir(out[:L], t[:L], i[:L])[1]
    assert abs(sir - float(g["sir_out"])) < 1e-4
    # the chunk-0 model inputs: [log(|Y0| + 1e-7), angle(Y0) - angle(Y1)] of the complex64
    # STFT of the float32 file data (sf.read(dtype='float32'), :257, :307-317)
    _, _, Y = O.stft(mix[:, :int(g["chunk"])], nperseg=int(g["n_fft"]),
                     noverlap=int(g["n_fft"]) // 2)
    assert Y.dtype == np.complex64
    np.testing.assert_allclose(np.log(np.abs(Y[0]) + 1e-7), g["chunk0_logmag"], atol=2e-6)
    d = np.angle(Y[0]) - np.angle(Y[1]) - g["chunk0_ipd"]
    assert (np.abs(d) <= 1e-5).all()


@pytest.mark.gpu
@pytest.mark.parametrize("trip", TRIPS)
def test_process_audio_file_matches_reference(gpu_device, tmp_path, trip):
    import torch
    from avz import tflite_pipeline, wavio
    from test_gpu_features import _check

    g = golden(f"tflite_{trip}.npz")
    mix, t, i = triple_f32(trip)
    inp, outp, model = tmp_path / "mixture.wav", tmp_path / "enhanced.wav", tmp_path / "m.tflite"
    wavio.write(str(inp), mix.T, 16000)  # int16 / 32768 values: exact through PCM-16
    model.write_bytes(b"")
    masks = torch.from_numpy(g["masks"]).to(gpu_device)
    seen = {}

    def mask_fn(feats):
        seen["f"] = feats[0].cpu().numpy()
        assert feats.shape == (masks.shape[0], 513, masks.shape[2], 2)
        return masks

    out = tflite_pipeline.process_audio_file(str(inp), str(outp), str(model), mask_fn=mask_fn)
    assert out.shape == g["out"].shape
    err = np.abs(out.astype(np.float64) - g["out"]).max()
    assert err <= WAVE_TOL, err
    L = min(len(out), len(t))
    sir = O.projection_sdr_sir(out[:L].astype(np.float64), t[:L], i[:L])[1]
    assert abs(sir - float(g["sir_out"])) <= SIR_TOL
    written, fs = wavio.read(str(outp))
    assert fs == 16000 and written.shape == out.shape
    assert np.abs(written - out).max() <= 1.0 / 32768 + 1e-7
    _, _, Y = O.stft(mix[:, :int(g["chunk"])], nperseg=1024, noverlap=512)
    _check(seen["f"][..., 0], seen["f"][..., 1], g["chunk0_logmag"], g["chunk0_ipd"], Y)


@pytest.mark.gpu
def test_process_audio_file_needs_model_and_mask_fn(gpu_device, tmp_path):
    from avz import tflite_pipeline
    with pytest.raises(FileNotFoundError):
        tflite_pipeline.process_audio_file("x.wav", str(tmp_path / "o.wav"),
                                           str(tmp_path / "absent.tflite"), mask_fn=lambda f: f)
    (tmp_path / "m.tflite").write_bytes(b"")
    with pytest.raises(RuntimeError):
        tflite_pipeline.process_audio_file("x.wav", str(tmp_path / "o.wav"),
                                           str(tmp_path / "m.tflite"))
