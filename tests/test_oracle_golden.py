"""Pin the CPU oracle to the reference: golden vectors made by running the reference
itself (tests/golden/make_golden.py). CPU only."""
import glob
import os

import numpy as np
import pytest
import scipy.signal

from conftest import GOLDEN, golden, triple_f32
from oracle import avz_oracle as O

FULL = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "full_*.npz")))
EXC = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "excerpt_*.npz")))


def test_fixture_inventory():
    assert len(FULL) == 12 and len(EXC) == 8


@pytest.mark.parametrize("n", [512, 1024])
def test_stft_matches_scipy(n):
    mix, tgt, _ = triple_f32("test", (1000, 23000))
    for x in (mix, tgt):
        f0, t0, Y0 = scipy.signal.stft(x, fs=16000, nperseg=n, noverlap=n // 2)
        f1, t1, Y1 = O.stft(x, fs=16000, nperseg=n, noverlap=n // 2)
        assert Y1.dtype == Y0.dtype == np.complex64
        assert Y1.shape == Y0.shape
        np.testing.assert_allclose(f1, f0)
        np.testing.assert_allclose(t1, t0)
        assert np.max(np.abs(Y1 - Y0)) <= 1e-6 * np.max(np.abs(Y0))


@pytest.mark.parametrize("n", [512, 1024])
@pytest.mark.parametrize("length", [1024, 1025, 1535, 4000, 64000])
def test_frame_count_and_istft_length(n, length):
    # scipy shrinks nperseg to the input length when L < nperseg (and then fails on
    # noverlap); the engine therefore rejects L < n_fft (AVZ_ERR_SHAPE).
    x = np.random.default_rng(length).standard_normal(length).astype(np.float32)
    _, _, Y = scipy.signal.stft(x, fs=16000, nperseg=n, noverlap=n // 2)
    assert Y.shape[-1] == O.n_frames(length, n, n // 2) == -(-length // (n // 2)) + 1
    _, xr0 = scipy.signal.istft(Y, fs=16000, nperseg=n, noverlap=n // 2)
    _, xr1 = O.istft(Y, fs=16000, nperseg=n, noverlap=n // 2)
    assert len(xr1) == len(xr0) == (Y.shape[-1] - 1) * (n // 2)
    np.testing.assert_allclose(xr1, xr0, atol=1e-12)


@pytest.mark.parametrize("name", FULL)
def test_oracle_debug_full_length(name):
    g = golden(name)
    trip = name.split("_")[1]
    mix, tgt, itf = triple_f32(trip)
    n, s = int(g["n_fft"]), float(g["sigma"])
    for fn in (O.oracle_debug_vec, O.oracle_debug_loop):
        out = fn(mix, tgt, itf, n_fft=n, hop=n // 2, sigma=s)
        assert len(out) == int(g["out_len"])
        np.testing.assert_allclose(out[::16], g["out_stride16"], atol=2e-7)
        np.testing.assert_allclose(out[:4096], g["out_head"], atol=2e-7)
        assert abs(np.sum(out ** 2) - float(g["sumsq"])) <= 1e-6 * float(g["sumsq"])
        L = min(len(out), len(tgt))
        _, sir = O.projection_sdr_sir(out[:L], tgt[:L], itf[:L])
        assert abs(sir - float(g["sir_out"])) < 1e-6
        if fn is O.oracle_debug_loop:
            continue
        _, sir_in = O.projection_sdr_sir(mix[0, :L], tgt[:L], itf[:L])
        assert abs(sir_in - float(g["sir_in"])) < 1e-6
        osinr, osir = O.osinr_osir(out[:L].astype(np.float64), tgt[:L].astype(np.float64),
                                   itf[:L].astype(np.float64))
        assert abs(osir - float(g["osir_out"])) < 1e-6 and abs(osinr - float(g["osinr_out"])) < 1e-6


@pytest.mark.parametrize("name", EXC)
def test_oracle_debug_excerpt_and_stages(name):
    g = golden(name)
    trip = name.split("_")[1]
    seg = g["seg"]
    mix, tgt, itf = triple_f32(trip, seg)
    n, s = int(g["n_fft"]), float(g["sigma"])
    out, st = O.oracle_debug_vec(mix, tgt, itf, n_fft=n, hop=n // 2, sigma=s, return_stages=True)
    np.testing.assert_allclose(out, g["out"], atol=2e-7)
    assert abs(st["peak"] - float(g["peak_raw"])) <= 1e-9 * float(g["peak_raw"])
    if "stage_bins" not in g:
        return
    bins = g["stage_bins"]
    np.testing.assert_allclose(st["Y"][:, bins, :], g["stage_Y_mix"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(st["S_t"][bins], g["stage_S_tgt"], atol=1e-9)
    np.testing.assert_allclose(st["S_i"][bins], g["stage_S_int"], atol=1e-9)
    sb = g["stage_solve_bins"]
    Rl = st["R"][sb] + s * np.eye(2)
    np.testing.assert_allclose(Rl, g["stage_R_loaded"], rtol=1e-12, atol=1e-18)
    # the reference's un-normalised solve, then its normalisation -> our weights
    w = g["stage_w_unnorm"]
    dv = g["stage_d"]
    w_ref = w / (np.sum(np.conj(dv) * w, axis=1, keepdims=True) + 1e-10)
    np.testing.assert_allclose(st["W"][sb], w_ref, rtol=1e-9)
    np.testing.assert_allclose(st["S_final"][bins], g["stage_S_final"], rtol=1e-9, atol=1e-15)


@pytest.mark.parametrize("trip", ["test", "set2"])
@pytest.mark.parametrize("n", [512, 1024])
def test_masked_mvdr_ipd(trip, n):
    g = golden(f"ipd_{trip}_n{n}.npz")
    mix, tgt, itf = triple_f32(trip)
    out, st = O.masked_mvdr_vec(mix, n_fft=n, hop=n // 2, return_stages=True)
    assert len(out) == int(g["out_len"])
    assert int(np.sum(st["mask"] < 1.0)) == int(g["mask_low_count"])
    np.testing.assert_allclose(out[::16], g["out_stride16"], atol=5e-6)
    L = min(len(out), len(tgt))
    _, sir = O.projection_sdr_sir(out[:L], tgt[:L], itf[:L])
    assert abs(sir - float(g["sir_out"])) < 1e-4
    ge = golden(f"ipd_excerpt_{trip}_n{n}.npz")
    mix_e, _, _ = triple_f32(trip, ge["seg"])
    np.testing.assert_allclose(O.masked_mvdr_vec(mix_e, n_fft=n, hop=n // 2), ge["out"], atol=5e-6)


REVERB = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "reverb_*_hp*.npz")))


def test_reverb_fixture_inventory():
    assert len(REVERB) == 6


@pytest.mark.parametrize("name", REVERB)
def test_oracle_reverb_full_length(name):
    """oracle_reverb.py:41-174 (IRM post-filter, --sigma/--hp) vs the reference run."""
    g = golden(name)
    trip = name.split("_")[1]
    mix, tgt, itf = triple_f32(trip)
    n, s, hp = int(g["n_fft"]), float(g["sigma"]), float(g["hp"])
    out, st = O.oracle_reverb_vec(mix, tgt, itf, n_fft=n, hop=n // 2, sigma=s, hp=hp,
                                  return_stages=True)
    assert len(out) == int(g["out_len"])
    np.testing.assert_allclose(out[::16], g["out_stride16"], atol=2e-7)
    np.testing.assert_allclose(out[:4096], g["out_head"], atol=2e-7)
    assert abs(st["peak"] - float(g["peak_raw"])) <= 1e-9 * float(g["peak_raw"])
    L = min(len(out), len(tgt))
    _, sir = O.projection_sdr_sir(out[:L], tgt[:L], itf[:L])
    assert abs(sir - float(g["sir_out"])) < 1e-6


def test_oracle_reverb_excerpt_spectrum():
    g = golden("reverb_excerpt_test_n512.npz")
    mix, tgt, itf = triple_f32("test", g["seg"])
    out, st = O.oracle_reverb_vec(mix, tgt, itf, n_fft=512, hop=256, sigma=float(g["sigma"]),
                                  hp=float(g["hp"]), return_stages=True)
    S = O.apply_weights(st["W"], st["Y"]) * st["gain"]
    np.testing.assert_allclose(S, g["S_final"], rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(out, g["out"], atol=2e-7)


def test_metric_vectors():
    g = golden("metrics_vectors.npz")
    sdr, sir = O.projection_sdr_sir(g["o"], g["t"], g["i"])
    osinr, osir = O.osinr_osir(g["o"], g["t"], g["i"])
    for a, b in ((sdr, g["sdr"]), (sir, g["sir"]), (osinr, g["osinr"]), (osir, g["osir"])):
        assert abs(a - float(b)) < 1e-10


def test_steering_vectors():
    g = golden("steering.npz")
    for j, (a, d) in enumerate(((90.0, 0.01), (40.0, 0.08), (130.0, 0.04))):
        np.testing.assert_allclose(O.steering_vectors(g["f"], a, d, 343.0), g["sv"][j], atol=1e-15)
        np.testing.assert_allclose(O.steering_vector(a, g["f"][9], d, 343.0)[:, 0], g["sv"][j][9],
                                   atol=1e-15)
