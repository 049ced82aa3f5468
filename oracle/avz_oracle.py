"""CPU restatement of the reference's mask-driven MVDR chain — TEST INFRASTRUCTURE ONLY.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg. The shipped path (``avz``) never calls into this module.

Every function cites the reference line it restates (paths relative to
/root/reference). The STFT/iSTFT live in a third-party dependency of the
reference (``scipy.signal``; unpinned ``"scipy"`` in pyproject.toml:25, 1.15.3 in
this image), restated here from scipy/signal/_spectral_py.py:

* stft  -> _spectral_helper (boundary='zeros' :2050-2058, padded :2060-2067,
  window cast :2083-2084, scale :2086-2094, _fft_helper :2158-2204,
  result.astype(outdtype) :2141).
* istft -> :1688-1729.

Two flavours of the pipeline are provided:

* ``*_loop``   — loop-faithful: the per-frequency Python loops of
  rt_av_zoom/core/oracle_debug.py:56-80 and masked_mvdr.py:92-124.
  This is the timed CPU baseline (``kind: "port"``).
* ``*_vec``    — vectorised numpy restatement (same math, broadcast over bins),
  used by tests as the fast checker.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------
# constants of the reference (rt_av_zoom/core/masked_mvdr.py:9-18,
# rt_av_zoom/core/oracle_debug.py:23-24, Final_pipeline/src/config.py:14-29)
# ----------------------------------------------------------------------------
FS = 16000
D_CORE = 0.01           # masked_mvdr.py:10 (imported by oracle_debug.py:11-19)
C_SOUND = 343.0         # masked_mvdr.py:11
ANGLE_TARGET = 90.0     # masked_mvdr.py:12, oracle_debug.py:23
SIGMA_ORACLE = 1.0      # oracle_debug.py:24
SIGMA_HEURISTIC = 1e-7  # masked_mvdr.py:16
FMIN_MVDR = 100.0       # oracle_debug.py:67, masked_mvdr.py:109


# ----------------------------------------------------------------------------
# window / framing
# ----------------------------------------------------------------------------
def hann_periodic(n: int) -> np.ndarray:
    """scipy.signal.get_window('hann', n) (fftbins=True => periodic), float64.

    Restates scipy/signal/windows/_windows.py general_cosine with a=[0.5, 0.5]
    on linspace(-pi, pi, n+1)[:-1] (the 'sym=False' extension/truncation).
    """
    fac = np.linspace(-np.pi, np.pi, n + 1)[:-1]
    return 0.5 + 0.5 * np.cos(fac)


def n_frames(length: int, n_fft: int, hop: int) -> int:
    """Frame count of scipy's stft with boundary='zeros', padded=True.

    Lp = L + 2*(N//2); nadd = (-(Lp-N) % H) % N (_spectral_py.py:2063);
    T = (Lp + nadd - N)//H + 1.
    """
    lp = length + 2 * (n_fft // 2)
    nadd = (-(lp - n_fft) % hop) % n_fft
    return (lp + nadd - n_fft) // hop + 1


def stft(x: np.ndarray, fs: float = FS, nperseg: int = 512, noverlap: int = 256):
    """Restatement of ``scipy.signal.stft(x, fs, nperseg=N, noverlap=O)`` as the
    reference calls it (oracle_debug.py:42-44, masked_mvdr.py:76,
    Final_pipeline/src/inference.py:198).

    Returns (f, t, Y) with Y [..., F, T] in complex64 (result.astype(outdtype)).
    """
    x = np.asarray(x)
    outdtype = np.result_type(x, np.complex64)
    n = nperseg
    hop = n - noverlap
    win = hann_periodic(n)
    win_c = win.astype(outdtype)                     # :2083-2084
    scale = np.sqrt(1.0 / win_c.sum() ** 2)          # :2092 ('spectrum'), :2094 sqrt for stft
    half = n // 2
    zeros = np.zeros(x.shape[:-1] + (half,), dtype=x.dtype)
    xe = np.concatenate((zeros, x, zeros), axis=-1)  # zero_ext
    nadd = (-(xe.shape[-1] - n) % hop) % n           # :2063
    xe = np.concatenate((xe, np.zeros(xe.shape[:-1] + (nadd,))), axis=-1)  # float64 promote
    frames = np.lib.stride_tricks.sliding_window_view(xe, n, axis=-1)[..., ::hop, :]
    res = win_c * frames                             # complex (fp64 x fp32-rounded window)
    res = np.fft.rfft(res.real, n=n)                 # _fft_helper onesided
    res = res * scale
    res = res.astype(outdtype)
    res = np.moveaxis(res, -1, -2)                   # [..., F, T]
    f = np.fft.rfftfreq(n, 1.0 / fs)
    t = np.arange(res.shape[-1]) * hop / float(fs)
    return f, t, res


def istft(S: np.ndarray, fs: float = FS, nperseg: int = 512, noverlap: int = 256):
    """Restatement of ``scipy.signal.istft(S, fs, nperseg=N, noverlap=O)``
    (_spectral_py.py:1688-1729): irfft, x win.sum(), windowed overlap-add,
    N/2 trim, divide by the OLA of win**2 where > 1e-10. Returns (t, x)."""
    S = np.asarray(S)
    n = nperseg
    hop = n - noverlap
    nseg = S.shape[-1]
    xsubs = np.fft.irfft(S, axis=-2, n=n)[..., :n, :]
    win = hann_periodic(n)
    if np.result_type(win, xsubs) != xsubs.dtype:
        win = win.astype(xsubs.dtype)
    xsubs = xsubs * win.sum()
    outlen = n + (nseg - 1) * hop
    x = np.zeros(S.shape[:-2] + (outlen,), dtype=xsubs.dtype)
    norm = np.zeros(outlen, dtype=xsubs.dtype)
    for ii in range(nseg):                           # :1708-1711 (per-frame OLA loop)
        x[..., ii * hop: ii * hop + n] += xsubs[..., ii] * win
        norm[ii * hop: ii * hop + n] += win ** 2
    x = x[..., n // 2: -(n // 2)]
    norm = norm[n // 2: -(n // 2)]
    x /= np.where(norm > 1e-10, norm, 1.0)
    return np.arange(x.shape[-1]) / float(fs), x.real


# ----------------------------------------------------------------------------
# masks, steering, covariance, solve
# ----------------------------------------------------------------------------
def steering_vector(angle_deg: float, f: float, d: float, c: float) -> np.ndarray:
    """rt_av_zoom/core/masked_mvdr.py:22-35 — (2,1) complex128."""
    theta = np.deg2rad(angle_deg)
    phi = 0.0
    tau1 = (d / 2) * np.cos(phi) * np.cos(theta - 0) / c
    tau2 = (d / 2) * np.cos(phi) * np.cos(theta - np.pi) / c
    omega = 2 * np.pi * f
    return np.array([[np.exp(-1j * omega * tau1)], [np.exp(-1j * omega * tau2)]], dtype=complex)


def steering_vectors(f_bins: np.ndarray, angle_deg: float, d: float, c: float) -> np.ndarray:
    """Vectorised form (tf_lite_version/inference.py:53-81): [F, 2] complex128."""
    theta = np.deg2rad(angle_deg)
    tau1 = (d / 2) * np.cos(theta) / c
    tau2 = (d / 2) * np.cos(theta - np.pi) / c
    omega = 2 * np.pi * np.asarray(f_bins, dtype=np.float64)
    return np.stack([np.exp(-1j * omega * tau1), np.exp(-1j * omega * tau2)], axis=-1)


def ibm_mask_noise(S_tgt: np.ndarray, S_int: np.ndarray) -> np.ndarray:
    """Oracle IBM, oracle_debug.py:49-53: 1.0 where |S_int| > |S_tgt| (strict)."""
    return np.where(np.abs(S_int) > np.abs(S_tgt), 1.0, 0.0)


def ipd_mask_noise(Y: np.ndarray) -> np.ndarray:
    """Heuristic phase mask, masked_mvdr.py:37-46: 1.0 where |angle(Y0)-angle(Y1)| > 0
    else 0.01 (angles of complex64 -> float32, difference in float32)."""
    pd = np.angle(Y[0]) - np.angle(Y[1])
    return np.where(np.abs(pd) > 0.0, 1.0, 0.01)


def covariance_loop(Y: np.ndarray, mask_noise: np.ndarray) -> np.ndarray:
    """Masked spatial covariance, oracle_debug.py:56-64 / masked_mvdr.py:92-102."""
    n_ch, n_f, _ = Y.shape
    R = np.zeros((n_f, n_ch, n_ch), dtype=complex)
    for fi in range(n_f):
        m_f = mask_noise[fi, :]
        Y_f = Y[:, fi, :]
        Yw = Y_f * np.sqrt(m_f)
        R[fi] = (Yw @ Yw.conj().T) / (np.sum(m_f) + 1e-6)
    return R


def covariance_vec(Y: np.ndarray, mask_noise: np.ndarray, weight_eps: float = 0.0) -> np.ndarray:
    """Same as covariance_loop, broadcast over bins (tf_lite_version/inference.py:103-127;
    weight_eps=1e-10 reproduces that variant's sqrt(mask + 1e-10))."""
    Yp = np.transpose(Y, (1, 0, 2))                    # F, M, T
    w = np.sqrt(mask_noise + weight_eps)[:, None, :]
    Yw = Yp * w
    R = np.einsum('fmt,fnt->fmn', Yw, Yw.conj())
    return R / (np.sum(mask_noise, axis=1)[:, None, None] + 1e-6)


def mvdr_weights_loop(R: np.ndarray, f: np.ndarray, sigma: float, angle: float, d: float,
                      c: float, fmin: float = FMIN_MVDR) -> np.ndarray:
    """Per-bin MVDR solve, oracle_debug.py:66-79: w = solve(R+sigma I, d);
    w /= (d^H w + 1e-10); LinAlgError -> [1, 0]; bins with f < fmin stay zero."""
    n_f = R.shape[0]
    W = np.zeros((n_f, 2), dtype=complex)
    for fi in range(n_f):
        if f[fi] < fmin:
            continue
        Rl = R[fi] + sigma * np.eye(2)
        dv = steering_vector(angle, f[fi], d, c)
        try:
            w = np.linalg.solve(Rl, dv)
            w /= (dv.conj().T @ w + 1e-10)
        except np.linalg.LinAlgError:
            w = np.array([[1], [0]])
        W[fi] = w[:, 0]
    return W


def mvdr_weights_vec(R: np.ndarray, f: np.ndarray, sigma: float, angle: float, d: float,
                     c: float, fmin: float = FMIN_MVDR) -> np.ndarray:
    """Closed-form 2x2 Hermitian solve, broadcast over bins (same result as the loop)."""
    dv = steering_vectors(f, angle, d, c)              # F, 2
    a = R[:, 0, 0] + sigma
    b = R[:, 0, 1]
    cc = R[:, 1, 0]
    e = R[:, 1, 1] + sigma
    det = a * e - b * cc
    ok = det != 0
    safe = np.where(ok, det, 1.0)
    w0 = (e * dv[:, 0] - b * dv[:, 1]) / safe
    w1 = (a * dv[:, 1] - cc * dv[:, 0]) / safe
    den = np.conj(dv[:, 0]) * w0 + np.conj(dv[:, 1]) * w1 + 1e-10
    W = np.stack([w0 / den, w1 / den], axis=-1)
    W[~ok] = np.array([1.0, 0.0])
    W[np.asarray(f) < fmin] = 0.0
    return W


def get_all_steering_vectors(f_bins: np.ndarray, angle_deg: float, d: float,
                             c: float) -> np.ndarray:
    """rt_av_zoom/core/tf_lite_version/inference.py:53-81: [F, 2, 1] complex128 far-field
    vectors exp(-1j 2 pi f tau_m), tau_1 = (d/2) cos(theta)/c, tau_2 = (d/2) cos(theta - pi)/c."""
    th = np.deg2rad(angle_deg)
    om = 2 * np.pi * np.asarray(f_bins)
    sv = np.stack([np.exp(-1j * om * ((d / 2) * np.cos(th) / c)),
                   np.exp(-1j * om * ((d / 2) * np.cos(th - np.pi) / c))], axis=0)
    return sv.T[:, :, None]


def batch_mvdr(Y: np.ndarray, mask: np.ndarray, f_bins, d_vectors: np.ndarray,
               sigma: float) -> np.ndarray:
    """rt_av_zoom/core/tf_lite_version/inference.py:85-179 restated with its dtypes: the
    noise weight 1 - mask (float32 for a float32 mask), Y * sqrt(w + 1e-10) and the
    covariance in complex64 (:103-117), / (sum w + 1e-6) (:121), + sigma I promotes to
    complex128 (:127-131), ONE batched solve whose LinAlgError sends every bin to
    w~ = [1, 0] (:139-153), w = w~ / (d^H w~ + 1e-10) (:159-163), S = w^H y (:169-175).
    f_bins is unused, as in the reference. Returns S [F, T] complex128."""
    Yp = np.transpose(Y, (1, 0, 2))
    mn = (1.0 - mask)[:, None, :]
    Yw = Yp * np.sqrt(mn + 1e-10)
    R = np.einsum('fmt,fnt->fmn', Yw, Yw.conj())
    R = R / (np.sum(mn, axis=2)[:, :, None] + 1e-6)
    R = R + sigma * np.eye(2)[None]
    try:
        wu = np.linalg.solve(R, d_vectors)
    except np.linalg.LinAlgError:
        wu = np.zeros_like(d_vectors)
        wu[:, 0, :] = 1.0
    den = np.matmul(np.transpose(d_vectors.conj(), (0, 2, 1)), wu) + 1e-10
    w = wu / den
    return np.matmul(np.transpose(w.conj(), (0, 2, 1)), Yp)[:, 0, :]


def hybrid_hard_null_bf(Y: np.ndarray, mask: np.ndarray, f_bins: np.ndarray,
                        d: float = 0.08) -> np.ndarray:
    """Final_pipeline/src/inference.py:28-98 as an operator: S[F, T] = w^H y with the
    loop-faithful per-bin weights (hybrid_weights_loop; bypass bins pass Y[0])."""
    W = hybrid_weights_loop(Y, mask, f_bins, d=d)
    return apply_weights(W, Y)


def apply_weights(W: np.ndarray, Y: np.ndarray) -> np.ndarray:
    """S[f,t] = w^H Y[:, f, t] (oracle_debug.py:80)."""
    return np.conj(W[:, 0])[:, None] * Y[0] + np.conj(W[:, 1])[:, None] * Y[1]


# ----------------------------------------------------------------------------
# end-to-end pipelines
# ----------------------------------------------------------------------------
def oracle_debug_loop(y_mix: np.ndarray, s_tgt: np.ndarray, s_int: np.ndarray, n_fft: int = 512,
                      hop: int = 256, sigma: float = SIGMA_ORACLE, d: float = D_CORE,
                      angle: float = ANGLE_TARGET, c: float = C_SOUND, fs: int = FS,
                      normalize: bool = True) -> np.ndarray:
    """rt_av_zoom/core/oracle_debug.py:27-97 minus file I/O (loop-faithful).

    Note oracle_debug passes noverlap=N_HOP; with N_HOP = N/2 that is a hop of N/2."""
    noverlap = n_fft - hop
    f, _, Y = stft(y_mix, fs=fs, nperseg=n_fft, noverlap=noverlap)
    _, _, S_t = stft(s_tgt, fs=fs, nperseg=n_fft, noverlap=noverlap)
    _, _, S_i = stft(s_int, fs=fs, nperseg=n_fft, noverlap=noverlap)
    mask = ibm_mask_noise(S_t, S_i)
    R = covariance_loop(Y, mask)
    n_f, n_t = Y.shape[1], Y.shape[2]
    S = np.zeros((n_f, n_t), dtype=complex)
    for fi in range(n_f):                               # oracle_debug.py:66-80
        if f[fi] < FMIN_MVDR:
            continue
        Rl = R[fi] + sigma * np.eye(2)
        dv = steering_vector(angle, f[fi], d, c)
        try:
            w = np.linalg.solve(Rl, dv)
            w /= (dv.conj().T @ w + 1e-10)
        except Exception:  # bare except in the reference (:78)
            w = np.array([[1], [0]])
        S[fi, :] = w.conj().T @ Y[:, fi, :]
    S_final = S * (1.0 - mask)                          # :84-90
    _, s_out = istft(S_final, fs=fs, nperseg=n_fft, noverlap=noverlap)
    if normalize:
        s_out = s_out / np.max(np.abs(s_out))           # :94
    return s_out


def oracle_debug_vec(y_mix, s_tgt, s_int, n_fft=512, hop=256, sigma=SIGMA_ORACLE, d=D_CORE,
                     angle=ANGLE_TARGET, c=C_SOUND, fs=FS, normalize=True, return_stages=False):
    """Vectorised restatement of oracle_debug.main (same math as the loop flavour)."""
    noverlap = n_fft - hop
    f, _, Y = stft(y_mix, fs=fs, nperseg=n_fft, noverlap=noverlap)
    _, _, S_t = stft(s_tgt, fs=fs, nperseg=n_fft, noverlap=noverlap)
    _, _, S_i = stft(s_int, fs=fs, nperseg=n_fft, noverlap=noverlap)
    mask = ibm_mask_noise(S_t, S_i)
    R = covariance_vec(Y, mask)
    W = mvdr_weights_vec(R, f, sigma, angle, d, c)
    S_final = apply_weights(W, Y) * (1.0 - mask)
    _, s_raw = istft(S_final, fs=fs, nperseg=n_fft, noverlap=noverlap)
    peak = np.max(np.abs(s_raw))
    s_out = s_raw / peak if normalize else s_raw
    if return_stages:
        return s_out, dict(Y=Y, S_t=S_t, S_i=S_i, mask=mask, R=R, W=W, S_final=S_final,
                           s_raw=s_raw, peak=peak, f=f)
    return s_out


def masked_mvdr_vec(y_mix, n_fft=512, hop=256, sigma=SIGMA_HEURISTIC, d=D_CORE,
                    angle=ANGLE_TARGET, c=C_SOUND, fs=FS, normalize=True, return_stages=False):
    """Heuristic IPD path, rt_av_zoom/core/masked_mvdr.py:50-132 minus I/O/plot:
    IPD noise mask, covariance, MVDR (sigma=1e-7), no post-filter,
    s /= (max|s| + 1e-6)."""
    noverlap = n_fft - hop
    f, _, Y = stft(y_mix, fs=fs, nperseg=n_fft, noverlap=noverlap)
    mask = ipd_mask_noise(Y)
    R = covariance_vec(Y, mask)
    W = mvdr_weights_vec(R, f, sigma, angle, d, c)
    S = apply_weights(W, Y)
    _, s_raw = istft(S, fs=fs, nperseg=n_fft, noverlap=noverlap)
    peak = np.max(np.abs(s_raw))
    s_out = s_raw / (peak + 1e-6) if normalize else s_raw
    if return_stages:
        return s_out, dict(Y=Y, mask=mask, R=R, W=W, S=S, s_raw=s_raw, peak=peak, f=f)
    return s_out


SIGMA_REVERB = 1e-3     # oracle_reverb.py:184 (--sigma default)


def irm_gain(S_t: np.ndarray, S_i: np.ndarray) -> np.ndarray:
    """Ideal-ratio-mask post-filter, oracle_reverb.py:143-156:
    sqrt(|S_t|^2 / (|S_t|^2 + |S_i|^2 + 1e-10)) in float32 (complex64 spectra)."""
    P_t = np.abs(S_t) ** 2
    P_i = np.abs(S_i) ** 2
    return np.sqrt(P_t / (P_t + P_i + 1e-10))


def oracle_reverb_vec(y_mix, s_tgt, s_int, n_fft=512, hop=256, sigma=SIGMA_REVERB, hp=100.0,
                      d=D_CORE, angle=ANGLE_TARGET, c=C_SOUND, fs=FS, normalize=True,
                      return_stages=False):
    """rt_av_zoom/core/oracle_reverb.py:41-174 minus file I/O (its input is the WPE
    output mixture_wpe.wav; WPE itself is out of scope): IBM (:84-86), covariance
    (:92-105), MVDR with diagonal loading sigma and the --hp cutoff, LinAlgError ->
    ones/2 (:113-138), IRM post-filter (:143-156), s /= max|s| + 1e-9 (:164)."""
    noverlap = n_fft - hop
    f, _, Y = stft(y_mix, fs=fs, nperseg=n_fft, noverlap=noverlap)
    _, _, S_t = stft(s_tgt, fs=fs, nperseg=n_fft, noverlap=noverlap)
    _, _, S_i = stft(s_int, fs=fs, nperseg=n_fft, noverlap=noverlap)
    mask = ibm_mask_noise(S_t, S_i)
    R = covariance_vec(Y, mask)
    f_hz = np.arange(Y.shape[1]) * fs / n_fft          # :114 freq_hz = f_idx * FS / N_FFT
    W = mvdr_weights_vec(R, f_hz, sigma, angle, d, c, fmin=hp)
    a = R[:, 0, 0] + sigma
    e = R[:, 1, 1] + sigma
    W[(a * e - R[:, 0, 1] * R[:, 1, 0] == 0) & (f_hz >= hp)] = 0.5   # :133-135 ones/n
    g = irm_gain(S_t, S_i)
    S_final = apply_weights(W, Y) * g
    _, s_raw = istft(S_final, fs=fs, nperseg=n_fft, noverlap=noverlap)
    peak = np.max(np.abs(s_raw))
    s_out = s_raw / (peak + 1e-9) if normalize else s_raw
    if return_stages:
        return s_out, dict(Y=Y, S_t=S_t, S_i=S_i, mask=mask, R=R, W=W, gain=g, s_raw=s_raw,
                           peak=peak, f=f)
    return s_out


def external_mask_vec(y_mix, mask_target, n_fft=1024, hop=512, sigma=1e-5, d=0.04,
                      angle=ANGLE_TARGET, c=C_SOUND, fs=FS, floor=0.05, weight_eps=0.0,
                      normalize=False):
    """External (neural) target mask path, full_audio_generating_pipeline/inference.py:88-118
    (process_chunk): noise mask 1-M, covariance, MVDR sigma=1e-5, post-filter max(M, 0.05).
    ``floor=None`` disables the post-filter."""
    noverlap = n_fft - hop
    f, _, Y = stft(y_mix, fs=fs, nperseg=n_fft, noverlap=noverlap)
    mask_n = 1.0 - mask_target
    R = covariance_vec(Y, mask_n, weight_eps)
    W = mvdr_weights_vec(R, f, sigma, angle, d, c)
    S = apply_weights(W, Y)
    if floor is not None:
        S = S * np.maximum(mask_target, floor)
    _, s_raw = istft(S, fs=fs, nperseg=n_fft, noverlap=noverlap)
    if normalize:
        return s_raw / np.max(np.abs(s_raw))
    return s_raw


def neural_deploy_vec(y: np.ndarray, masks, chunk: int = 32000, n_fft: int = 1024,
                      d: float = 0.04, sigma: float = 1e-5) -> np.ndarray:
    """full_audio_generating_pipeline/inference.py:120-167 (main_deploy minus file I/O and
    the model): y [S, 2]; masks[c] is the target mask of chunk c (the U-Net output);
    each chunk through external_mask_vec (process_chunk, :88-118), the first
    min(len(out), chunk) samples overlap-added at c * chunk/2, divided by the count."""
    hop = chunk // 2
    S = y.shape[0]
    out_buf = np.zeros(S + chunk)
    norm_buf = np.zeros(S + chunk)
    for c in range(int(np.ceil(S / hop))):
        seg = y[c * hop:c * hop + chunk]
        if len(seg) < chunk:
            seg = np.pad(seg, ((0, chunk - len(seg)), (0, 0)))
        o = external_mask_vec(seg.T, masks[c], n_fft=n_fft, hop=n_fft // 2, sigma=sigma, d=d)
        L = min(len(o), chunk)
        out_buf[c * hop:c * hop + L] += o[:L]
        norm_buf[c * hop:c * hop + L] += 1.0
    norm_buf[norm_buf == 0] = 1.0
    return out_buf[:S] / norm_buf[:S]


def process_audio_file_vec(y: np.ndarray, masks, chunk: int = 32000, n_fft: int = 1024,
                           d: float = 0.04, c: float = C_SOUND, sigma: float = 1e-5,
                           fs: int = FS) -> np.ndarray:
    """rt_av_zoom/core/tf_lite_version/inference.py:245-391 (process_audio_file minus file
    I/O, timing prints and the TFLite model): y [S, 2]; masks[i] the target mask of chunk i
    (TFLiteBeamformer.predict_mask's output, :300). Chunks of ``chunk`` samples every
    chunk // 2, ceil(S / hop) of them, zero-padded tail (:269-289); stft (:293); batch_mvdr
    with the module's steering vectors (:320-327); S * max(M, 0.05) and the whole istft output
    (:341-345, 32256 samples for a 32000-sample chunk) overlap-added at the chunk start,
    clipped at the end of the buffer, with a per-sample count (:349-355); out / count
    (count 0 -> 1) and peak normalisation + 1e-9 (:361-365)."""
    hop_c = chunk // 2
    S = y.shape[0]
    out_buf = np.zeros(S)
    norm_buf = np.zeros(S)
    for i in range(int(np.ceil(S / hop_c))):
        start = i * hop_c
        seg = y[start:start + chunk]
        if len(seg) < chunk:
            seg = np.pad(seg, ((0, chunk - len(seg)), (0, 0)))
        f_bins, _, Y = stft(seg.T, fs=fs, nperseg=n_fft, noverlap=n_fft // 2)
        M = np.asarray(masks[i])
        mf, mt = min(M.shape[0], Y.shape[1]), min(M.shape[1], Y.shape[2])
        M, Y, fv = M[:mf, :mt], Y[:, :mf, :mt], f_bins[:mf]
        S_out = batch_mvdr(Y, M, fv, get_all_steering_vectors(fv, ANGLE_TARGET, d, c), sigma)
        _, xo = istft(S_out * np.maximum(M, 0.05), fs=fs, nperseg=n_fft, noverlap=n_fft // 2)
        w = min(len(xo), S - start)
        out_buf[start:start + w] += xo[:w]
        norm_buf[start:start + w] += 1.0
    norm_buf[norm_buf == 0] = 1.0
    final = out_buf / norm_buf
    return final / (np.max(np.abs(final)) + 1e-9)


# ----------------------------------------------------------------------------
# Final_pipeline: hybrid hard-null beamformer + 2-s chunked overlap-add driver
# ----------------------------------------------------------------------------
D_FINAL = 0.08          # Final_pipeline/src/config.py:29 (MIC_DIST)
WIN_SIZE = 32000        # Final_pipeline/src/config.py:17 (chunk), hop = WIN_SIZE // 2
BYPASS_HZ = 200.0       # Final_pipeline/src/inference.py:50
COND_MAX = 10.0         # Final_pipeline/src/inference.py:80


def steering_vector_phase_norm(f: float, angle_deg: float = ANGLE_TARGET, d: float = D_FINAL,
                               c: float = C_SOUND) -> np.ndarray:
    """Final_pipeline/src/inference.py:16-26: far-field vector divided by (v[0] + 1e-10)."""
    th = np.deg2rad(angle_deg)
    om = 2 * np.pi * f
    v = np.array([[np.exp(-1j * om * ((d / 2) * np.cos(th) / c))],
                  [np.exp(-1j * om * ((d / 2) * np.cos(th - np.pi) / c))]])
    return v / (v[0] + 1e-10)


def hybrid_weights_loop(Y: np.ndarray, mask: np.ndarray, f_bins: np.ndarray,
                        d: float = D_FINAL, bypass_hz: float = BYPASS_HZ,
                        cond_max: float = COND_MAX) -> np.ndarray:
    """Per-bin weights of Final_pipeline/src/inference.py:28-98 (hybrid_hard_null_bf),
    loop-faithful: complex64 noise covariance (:57-60), LAPACK eigh principal vector
    phase-normalised to mic 0 (:63-67), cond of [v_tgt, v_int] (:77), delay-and-sum
    fallback or solve C^H w = [1, 0] (:79-91). Returns W [F, 2] complex128; the bypass
    bins (f < bypass_hz, :50-52) get w = [1, 0] (S = Y0)."""
    F = Y.shape[1]
    m_int = 1.0 - mask
    W = np.zeros((F, 2), dtype=np.complex128)
    e1 = np.array([[1], [0]], dtype=np.complex64)
    for k in range(F):
        fk = f_bins[k]
        if fk < bypass_hz:
            W[k] = [1.0, 0.0]
            continue
        Yk = Y[:, k, :]
        mk = m_int[k, :]
        R = (Yk * mk) @ Yk.conj().T / (np.sum(mk) + 1e-6)
        _, vecs = np.linalg.eigh(R)
        v_int = vecs[:, -1].reshape(2, 1)
        v_int = v_int / (v_int[0] / (np.abs(v_int[0]) + 1e-10))
        v_tgt = steering_vector_phase_norm(fk, ANGLE_TARGET, d, C_SOUND)
        C = np.column_stack((v_tgt, v_int))
        if np.linalg.cond(C) > cond_max:
            w = v_tgt / 2
        else:
            try:
                w = np.linalg.solve(C.conj().T, e1)
            except np.linalg.LinAlgError:
                w = v_tgt / 2
        W[k] = w[:, 0]
    return W


def hybrid_weights_vec(Y: np.ndarray, mask: np.ndarray, f_bins: np.ndarray,
                       d: float = D_FINAL, bypass_hz: float = BYPASS_HZ,
                       cond_max: float = COND_MAX) -> np.ndarray:
    """Closed-form fp64 form of hybrid_weights_loop (the engine's per-bin algebra):
    principal eigenvector of the 2x2 Hermitian R, cond_2 = sigma_max^2 / |det C|,
    w = [conj v1, -conj v0] / conj(det C). A bin whose eigenvector has v[0] == 0 (where
    the reference divides by zero) takes the delay-and-sum fallback."""
    Yd = Y.astype(np.complex128)
    m = (1.0 - mask).astype(np.float64)
    nrm = m.sum(axis=1) + 1e-6
    a = np.einsum("ft,ft->f", m, np.abs(Yd[0]) ** 2) / nrm
    e = np.einsum("ft,ft->f", m, np.abs(Yd[1]) ** 2) / nrm
    b = np.einsum("ft,ft->f", m, Yd[0] * Yd[1].conj()) / nrm
    lam = 0.5 * (a + e) + np.sqrt((0.5 * (a - e)) ** 2 + np.abs(b) ** 2)
    u0 = np.where(a >= e, lam - e + 0j, b)
    u1 = np.where(a >= e, b.conj(), lam - a + 0j)
    un = np.sqrt(np.abs(u0) ** 2 + np.abs(u1) ** 2)
    with np.errstate(divide="ignore", invalid="ignore"):
        u0, u1 = u0 / un, u1 / un
        a0 = np.abs(u0)
        v0 = a0 + 1e-10 + 0j
        v1 = u1 * u0.conj() * (a0 + 1e-10) / a0 ** 2
    vt = np.stack([steering_vector_phase_norm(fk, ANGLE_TARGET, d, C_SOUND)[:, 0]
                   for fk in f_bins])
    t0, t1 = vt[:, 0], vt[:, 1]
    det = t0 * v1 - v0 * t1
    p = np.abs(t0) ** 2 + np.abs(t1) ** 2
    q = np.abs(v0) ** 2 + np.abs(v1) ** 2
    r = t0.conj() * v0 + t1.conj() * v1
    smax2 = 0.5 * (p + q) + np.sqrt((0.5 * (p - q)) ** 2 + np.abs(r) ** 2)
    ok = np.isfinite(v1) & (a0 > 0) & (np.abs(det) > 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        ok &= smax2 <= cond_max * np.abs(det)
        W = np.where(ok[:, None], np.stack([v1.conj(), -v0.conj()], axis=1) / det.conj()[:, None],
                     vt / 2)
    W[f_bins < bypass_hz] = [1.0, 0.0]
    return W


def enhance_chunked(y: np.ndarray, mask_fn, bf="loop", n_fft: int = 1024, chunk: int = WIN_SIZE,
                    fs: int = FS, d: float = D_FINAL):
    """Final_pipeline/src/inference.py:160-237 (enhance_audio minus file I/O): y [S, 2]
    float32; ``mask_fn(c, start, chunk_samples [chunk, 2]) -> M [F, T]`` target probability
    (stands in for TFLiteBeamformer.predict_mask). Chunks of ``chunk`` samples every
    chunk // 2 with a zero-padded tail (:179-188), hybrid weights, x M post-filter (:219),
    iSTFT, time-domain overlap-add / count (:226-229), peak normalisation + 1e-9 (:236)."""
    hop_c = chunk // 2
    L = len(y)
    out = np.zeros(L)
    cnt = np.zeros(L)
    wfn = hybrid_weights_loop if bf == "loop" else hybrid_weights_vec
    for c in range(int(np.ceil(L / hop_c))):
        start = c * hop_c
        seg = y[start:start + chunk]
        if len(seg) < chunk:
            seg = np.pad(seg, ((0, chunk - len(seg)), (0, 0)))
        f, _, Y = stft(seg.T, fs=fs, nperseg=n_fft, noverlap=n_fft // 2)
        M = mask_fn(c, start, seg)
        W = wfn(Y, M, f, d=d)
        S = np.einsum("fm,mft->ft", W.conj(), Y) * M
        _, xo = istft(S, fs=fs, nperseg=n_fft, noverlap=n_fft // 2)
        n = min(len(xo), L - start)
        out[start:start + n] += xo[:n]
        cnt[start:start + n] += 1.0
    final = out / np.maximum(cnt, 1.0)
    return final / (np.max(np.abs(final)) + 1e-9)


def mask_features(y2: np.ndarray, n_fft: int = 1024, layout: str = "unet") -> np.ndarray:
    """Mask-model inputs of a [2, S] mic pair, float32 as numpy computes them:
    "unet"   -> [2, F, T]  log(|Y0| + 1e-7), angle(Y0) - angle(Y1)
                (full_audio_generating_pipeline/inference.py:90-94);
    "tflite" -> [F, T, 4]  + sin/cos of the IPD and linspace(0, 1, F)
                (Final_pipeline/src/inference.py:198-203, 117-128)."""
    _, _, Y = stft(y2, nperseg=n_fft, noverlap=n_fft // 2)
    lm = np.log(np.abs(Y[0]) + 1e-7)
    ipd = np.angle(Y[0]) - np.angle(Y[1])
    if layout == "unet":
        return np.stack([lm, ipd])
    F, T = lm.shape
    fm = np.tile(np.linspace(0, 1, F, dtype=np.float32)[:, None], (1, T))
    return np.stack([lm, np.sin(ipd), np.cos(ipd), fm], axis=-1)


def srp_scan(y2: np.ndarray, n_fft: int = 512, d: float = D_CORE, c: float = C_SOUND,
             fs: int = FS, f_lo: float = 200.0, f_hi: float = 4000.0, n_angles: int = 181):
    """scripts/debug_srp.py:46-62: steered response power over linspace(0, 180, 181),
    summed over 200 <= f <= 4000 Hz and all frames, in dB relative to the maximum."""
    f, _, Y = stft(y2, fs=fs, nperseg=n_fft, noverlap=n_fft // 2)
    angles = np.linspace(0, 180, n_angles)
    sel = (f >= f_lo) & (f <= f_hi)
    P = []
    for a in angles:
        th = np.deg2rad(a)
        t1 = (d / 2) * np.cos(0) * np.cos(th - 0) / c
        t2 = (d / 2) * np.cos(0) * np.cos(th - np.pi) / c
        om = 2 * np.pi * f[sel]
        dv = np.stack([np.exp(-1j * om * t1), np.exp(-1j * om * t2)])       # [2, F']
        out = np.einsum("mf,mft->ft", dv.conj(), Y[:, sel, :])
        P.append(np.sum(np.abs(out) ** 2))
    P = 10 * np.log10(np.array(P))
    return angles, P - P.max()


def chunk_target_mask(tgt: np.ndarray, itf: np.ndarray, start: int, chunk: int = WIN_SIZE,
                      n_fft: int = 1024) -> np.ndarray:
    """Oracle target mask |S_t| >= |S_i| of one driver chunk (the stand-in for the absent
    TFLite mask model used by the golden fixtures, tests/golden/make_golden.py)."""
    st = np.pad(tgt[start:start + chunk], (0, max(0, chunk - len(tgt[start:start + chunk]))))
    si = np.pad(itf[start:start + chunk], (0, max(0, chunk - len(itf[start:start + chunk]))))
    _, _, St = stft(st, nperseg=n_fft, noverlap=n_fft // 2)
    _, _, Si = stft(si, nperseg=n_fft, noverlap=n_fft // 2)
    return (np.abs(St) >= np.abs(Si)).astype(np.float32)


# ----------------------------------------------------------------------------
# metrics
# ----------------------------------------------------------------------------
def projection_sdr_sir(output, target, interf):
    """scripts/run_metrics.py:6-36 (calculate_metrics_manual) -> (sdr, sir) in dB."""
    eps = 1e-10
    o = output / (np.linalg.norm(output) + eps)
    t = target / (np.linalg.norm(target) + eps)
    i = interf / (np.linalg.norm(interf) + eps)
    alpha = np.dot(o, t)
    beta = np.dot(o, i)
    e_t = alpha * t
    e_i = beta * i
    e_a = o - e_t - e_i
    p_t = np.sum(e_t ** 2)
    p_i = np.sum(e_i ** 2) + 1e-10
    p_n = np.sum(e_a ** 2) + 1e-10
    return 10 * np.log10(p_t / (p_i + p_n)), 10 * np.log10(p_t / p_i)


def osinr_osir(output, target, interf):
    """Final_pipeline/src/metrics.py:102-123 (calculate_osnr_osir) -> (OSINR, OSIR)."""
    eps = 1e-10
    t = target / (np.linalg.norm(target) + eps)
    i = interf / (np.linalg.norm(interf) + eps)
    alpha = np.dot(output, t)
    beta = np.dot(output, i)
    e_t = alpha * t
    e_i = beta * i
    e_n = output - e_t - e_i
    p_t = np.sum(e_t ** 2)
    p_i = np.sum(e_i ** 2)
    p_n = np.sum(e_n ** 2)
    return 10 * np.log10(p_t / (p_i + p_n + eps)), 10 * np.log10(p_t / (p_i + eps))
