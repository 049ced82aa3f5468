"""Host-side pieces that need no GPU: WAV I/O conventions, batched device-agnostic
metrics (run on CPU tensors here) vs the reference's metric vectors, the synthetic
scene generator's conventions, and the reference-surface constants."""
import numpy as np
import torch

from conftest import golden
from oracle import avz_oracle as O


def test_wav_roundtrip_matches_int16_mapping(tmp_path):
    from avz import wavio
    rng = np.random.default_rng(0)
    x = np.clip(rng.standard_normal((1000, 2)) * 0.3, -1, 0.999).astype(np.float32)
    p = str(tmp_path / "a.wav")
    wavio.write(p, x, 16000)
    y, fs = wavio.read(p)
    assert fs == 16000 and y.shape == (1000, 2) and y.dtype == np.float32
    assert np.max(np.abs(y - x)) <= 0.5 / 32768 + 1e-7
    m, _ = wavio.read(p[:-5] + "a.wav")
    g = golden("inputs_test.npz")
    wavio.write(str(tmp_path / "t.wav"), g["tgt"][:500] / 32768.0, 16000)
    t, _ = wavio.read(str(tmp_path / "t.wav"))
    np.testing.assert_array_equal(t, (g["tgt"][:500].astype(np.float64) / 32768).astype(np.float32))


def test_batched_metrics_match_reference_vectors():
    from avz import metrics
    g = golden("metrics_vectors.npz")
    o, t, i = (torch.from_numpy(g[k])[None] for k in ("o", "t", "i"))
    sdr, sir = metrics.calculate_metrics_manual(o, t, i)
    osinr, osir = metrics.calculate_osnr_osir(o, t, i)
    for a, b in ((sdr, g["sdr"]), (sir, g["sir"]), (osinr, g["osinr"]), (osir, g["osir"])):
        assert abs(float(a[0]) - float(b)) < 1e-9


def test_metrics_ragged_lengths_mask():
    from avz import metrics
    rng = np.random.default_rng(1)
    o, t, i = rng.standard_normal((3, 2, 800))
    L = [800, 500]
    sdr, sir = metrics.calculate_metrics_manual(torch.from_numpy(o), torch.from_numpy(t),
                                                torch.from_numpy(i), torch.tensor(L))
    for b in range(2):
        ref = O.projection_sdr_sir(o[b, :L[b]], t[b, :L[b]], i[b, :L[b]])
        assert abs(float(sdr[b]) - ref[0]) < 1e-9 and abs(float(sir[b]) - ref[1]) < 1e-9


def test_synthetic_scene_conventions():
    from avz import synth
    mix, tgt, itf = synth.make_scene(5, n_samples=16000, n_interferers=2)
    assert mix.shape == (2, 16000) and mix.dtype == np.float32
    assert abs(np.max(np.abs(mix)) - 1.0) < 1e-6            # shared peak normalisation
    # SIR 0 dB on mic 1 between the refs (simulation.py:167-179)
    assert abs(10 * np.log10(np.mean(tgt.astype(np.float64) ** 2) /
                             np.mean(itf.astype(np.float64) ** 2))) < 1e-4
    m2, t2, i2 = synth.make_scene(5, n_samples=16000, n_interferers=2)
    np.testing.assert_array_equal(mix, m2)                   # deterministic per index
    # target at broadside: identical on both mics before noise -> mic difference is
    # interference + noise only
    d = mix[0] - mix[1]
    assert np.mean(d.astype(np.float64) ** 2) < np.mean(mix[0].astype(np.float64) ** 2)


def test_reference_surface_constants_and_steering():
    from avz import masked_mvdr, oracle_debug
    assert (masked_mvdr.FS, masked_mvdr.D, masked_mvdr.C, masked_mvdr.SIGMA,
            masked_mvdr.N_FFT, masked_mvdr.N_HOP) == (16000, 0.01, 343.0, 1e-7, 512, 256)
    assert oracle_debug.SIGMA == 1 and oracle_debug.OUTDIR.startswith("simulation_results/")
    g = golden("steering.npz")
    for j, (a, d) in enumerate(((90.0, 0.01), (40.0, 0.08), (130.0, 0.04))):
        for k in (0, 7, 100, 512):
            np.testing.assert_allclose(masked_mvdr.get_steering_vector(a, g["f"][k], d, 343.0)[:, 0],
                                       g["sv"][j][k], atol=1e-15)


def test_report_format_matches_reference():
    """report.txt / batch_metrics.csv formats (Final_pipeline/src/metrics.py:16-44,
    166-182) reproduced from the metric values; the golden was written by the reference's
    own evaluate_run."""
    from avz import metrics
    g = golden("report_test.npz")
    ref = str(g["report"]).splitlines()
    m = dict(sir_b=-4.48, sinr_b=-4.48, sir_s=24.07, sinr_s=9.41, stoi=0.0, pesq_wb=0.0,
             pesq_nb=0.0)
    ts = ref[1].split("Date: ")[1]
    assert metrics.format_report("golden_run", m, ts).splitlines() == ref
    row = metrics.csv_row("golden_run", m)
    assert ",".join(row[k] for k in metrics.CSV_HEADER) == str(g["csv"]).splitlines()[1]
