"""GPU parity of the oracle_reverb path (rt_av_zoom/core/oracle_reverb.py:41-174):
oracle IBM covariance, MVDR with --sigma / --hp, ideal-ratio-mask post-filter
(AVZ_PF_IRM), singular bins -> ones/2, s /= max|s| + 1e-9. Against the reference run on
the bundled triples (tests/golden/reverb_*.npz, make_golden.py gen_reverb). Tolerances as
test_gpu_parity.py: waveform max-abs <= 1e-4, SIR |delta| <= 0.01 dB."""
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
REVERB = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "reverb_*_hp*.npz")))


@pytest.fixture(scope="module")
def orv(gpu_device):
    from avz import oracle_reverb
    return oracle_reverb


def sir(out, tgt, itf):
    L = min(len(out), len(tgt))
    return O.projection_sdr_sir(out[:L].astype(np.float64), tgt[:L], itf[:L])[1]


@pytest.mark.parametrize("name", REVERB)
def test_reverb_full_length_vs_reference(orv, name):
    g = golden(name)
    trip = name.split("_")[1]
    mix, tgt, itf = triple_f32(trip)
    n, s, hp = int(g["n_fft"]), float(g["sigma"]), float(g["hp"])
    out = orv.enhance(mix, tgt, itf, sigma=s, hp_cutoff=hp, n_fft=n).astype(np.float64)
    assert len(out) == int(g["out_len"])
    assert np.max(np.abs(out[::16] - g["out_stride16"])) <= WAVE_TOL
    assert np.max(np.abs(out[:4096] - g["out_head"])) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - float(g["sir_out"])) <= SIR_TOL


def test_reverb_excerpt_full_waveform(orv):
    g = golden("reverb_excerpt_test_n512.npz")
    mix, tgt, itf = triple_f32("test", g["seg"])
    out = orv.enhance(mix, tgt, itf, sigma=float(g["sigma"]), hp_cutoff=float(g["hp"]),
                      n_fft=512).astype(np.float64)
    ref = g["out"].astype(np.float64)
    assert len(out) == len(ref)
    assert np.max(np.abs(out - ref)) <= WAVE_TOL
    assert abs(sir(out, tgt, itf) - sir(ref, tgt, itf)) <= SIR_TOL


def test_reverb_main_file_mirror(orv, tmp_path):
    """main(args) reads mixture_wpe.wav + references and writes output_oracle_reverb.wav."""
    from avz import wavio
    mix, tgt, itf = triple_f32("test", (20000, 52000))   # int16/32768: writes back exactly
    wavio.write(str(tmp_path / "mixture_wpe.wav"), mix.T, 16000)
    wavio.write(str(tmp_path / "target_reference.wav"), tgt, 16000)
    wavio.write(str(tmp_path / "interference_reference.wav"), itf, 16000)

    class Args:
        outdir, sigma, hp = str(tmp_path), 1e-3, 100.0
    out = orv.main(Args)
    assert (tmp_path / "output_oracle_reverb.wav").exists()
    ref = O.oracle_reverb_vec(mix, tgt, itf, n_fft=512, hop=256, sigma=1e-3, hp=100.0)
    assert np.max(np.abs(out.astype(np.float64) - ref)) <= WAVE_TOL
    assert orv.main(type("A", (), {"outdir": str(tmp_path / "absent"), "sigma": 1.0,
                                   "hp": 100.0})) is None


@pytest.mark.parametrize("fallback,expect", [("mean", (0.5, 0.5)), ("mic0", (1.0, 0.0))])
def test_singular_fallback_weights(gpu_device, fallback, expect):
    """A bin whose loaded covariance is singular (no noise-dominated frame, sigma = 0)
    takes ones/2 (oracle_reverb.py:133-135) or [1, 0] (oracle_debug.py:78-79)."""
    import avz
    rng = np.random.default_rng(3)
    S, n = 8000, 512
    x = rng.standard_normal(S).astype(np.float32)
    mix = np.stack([x, x])
    plan = avz.MVDRPlan(n_fft=n, sigma=0.0, fmin_hz=100.0, mask="ibm", postfilter="irm",
                        singular_fallback=fallback, normalize="none", max_batch=1, max_samples=S)
    F = n // 2 + 1
    w = torch.zeros((1, F, 4), dtype=torch.float32, device=gpu_device)
    d = lambda a: torch.from_numpy(a).to(gpu_device)[None]  # noqa: E731
    out, _ = plan.run(d(mix), ref_tgt=d(x), ref_int=d(np.zeros_like(x)), w_out=w)
    torch.cuda.synchronize()
    w = w[0].cpu().numpy()
    f = np.fft.rfftfreq(n, 1 / 16000)
    hi = f >= 100.0
    np.testing.assert_array_equal(w[hi, 0], expect[0])
    np.testing.assert_array_equal(w[hi, 2], expect[1])
    np.testing.assert_array_equal(w[hi][:, [1, 3]], 0.0)
    np.testing.assert_array_equal(w[~hi], 0.0)
    # IRM gain ~ 1 (no interference): the output is the weighted mic sum, high-passed
    ref = O.oracle_reverb_vec(mix, x, np.zeros_like(x), n_fft=n, hop=n // 2, sigma=0.0,
                              hp=100.0, normalize=False) if fallback == "mean" else None
    if ref is not None:
        got = out[0, :len(ref)].cpu().numpy().astype(np.float64)
        assert np.max(np.abs(got - ref)) <= 1e-4 * np.max(np.abs(ref))
