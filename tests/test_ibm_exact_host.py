"""Host-side pins of the reference-exact IBM path (avz_ibm_exact.hpp).

The device recomputes an uncertified decision as the reference forms it
(rt_av_zoom/core/oracle_debug.py:42-53): fp64 spectra of the two references, scaled by
1/sum(win), rounded to complex64, compared through numpy's complex64 magnitude. These tests
pin the three facts that restatement relies on, on the CPU:
  * numpy's np.abs of complex64 is larger * sqrt(fma(r, r, 1)), r = smaller / larger, in fp32
    (its SIMD loop; not hypotf) -- the formula np_abs_c64 evaluates;
  * scipy's STFT scale 1/sum(win) is an exact power of two at both FFT sizes, so it cannot move
    a complex64 rounding and the device may leave it out;
  * the library's fp32 window table (avz_ibm_window) is bitwise scipy's window as the
    reference's stft casts it.
"""
import ctypes as ct

import numpy as np
import pytest
import scipy.signal

from oracle import avz_oracle as O


def np_abs_c64_model(z):
    """The device's np_abs_c64, restated in numpy (fp32 ops, the fma in fp64 = one rounding)."""
    f = np.float32
    a, b = np.abs(z.real).astype(f), np.abs(z.imag).astype(f)
    lg, sm = np.maximum(a, b), np.minimum(a, b)
    with np.errstate(all="ignore"):
        r = (sm / lg).astype(f)
        q = (r.astype(np.float64) ** 2 + 1.0).astype(f)
        out = (lg * np.sqrt(q)).astype(f)
    return np.where(lg == 0, f(0), out)


def test_numpy_complex64_abs_formula():
    rng = np.random.default_rng(7)
    n = 400_000
    parts = []
    for scale in (1.0, 1e-18, 1e18, 1e-36):
        re = rng.standard_normal(n) * scale
        im = rng.standard_normal(n) * scale * rng.uniform(0, 3, n)
        parts.append((re + 1j * im).astype(np.complex64))
    # ties, zeros, one-sided and subnormal operands
    edge = np.array([0, 1e-45, 1e-45j, 3 + 4j, 1e-40 + 1e-40j, 1e30 + 1e30j, 1e-20 + 1e20j,
                     -0.0 - 0.0j, 1 + 1j, -2 - 2j], np.complex64)
    z = np.concatenate(parts + [edge])
    got = np.abs(z)
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got, np_abs_c64_model(z))
    # and on the reference's own STFT layout (non-contiguous complex64 from scipy.signal.stft)
    x = rng.standard_normal(20000).astype(np.float32)
    _, _, S = scipy.signal.stft(x, fs=16000, nperseg=1024, noverlap=512)
    assert not S.flags["C_CONTIGUOUS"]
    np.testing.assert_array_equal(np.abs(S), np_abs_c64_model(S))


@pytest.mark.parametrize("n", [512, 1024])
def test_stft_scale_is_a_power_of_two(n):
    win_c = O.hann_periodic(n).astype(np.complex64)
    scale = np.sqrt(1.0 / win_c.sum() ** 2)
    assert scale.imag == 0 and float(scale.real) == 2.0 / n


@pytest.mark.parametrize("n", [512, 1024])
def test_library_window_is_the_reference_window(n):
    from avz._lib import lib
    buf = (ct.c_float * n)()
    assert lib.avz_ibm_window(n, buf) == 0
    got = np.frombuffer(buf, dtype=np.float32)
    want = scipy.signal.get_window("hann", n).astype(np.float32)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, O.hann_periodic(n).astype(np.float32))
    assert lib.avz_ibm_window(768, buf) < 0
