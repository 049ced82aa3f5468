"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only in the build container (needs /root/reference, read-only). Nothing under
tests/, bench.py or smoke() reads /root/reference at run time: they read the .npz
files this script writes.

How the reference is run:
* ``soundfile`` (libsndfile) is not installed. A stand-in module is injected whose
  ``read`` decodes the bundled int16 WAVs with scipy.io.wavfile and divides by 32768
  (libsndfile's int16 -> float mapping), and whose ``write`` captures the float array
  instead of quantising to PCM_16. It touches only file I/O, never the arithmetic.
* matplotlib is forced to the Agg backend (masked_mvdr.main saves a PNG).
* oracle_debug.main() reads a hard-coded OUTDIR (oracle_debug.py:25); we chdir to a
  temp dir holding that folder. N_FFT/N_HOP/SIGMA are module globals we patch.
* Intermediates are captured by wrapping scipy.signal.stft/istft and
  numpy.linalg.solve for the duration of one reference call.

Final_pipeline/src/inference.py imports tensorflow at module level; an empty stand-in
module is injected (only TFLiteBeamformer uses it, and that class is replaced by
_MaskFeeder below because the .tflite model file is absent).

Usage:  python tests/golden/make_golden.py [hybrid] [srp] [report] [reverb] [neural] [world]
        [spectral] [tflite]
        (writes tests/golden/*.npz)
"""
from __future__ import annotations

import contextlib
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np
import scipy.io.wavfile as wavfile
import scipy.signal

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
INPUTS = os.path.join(REF, "data", "inputs")

TRIPLES = {
    "test": ("test_mixture", "test_target_ref", "test_interferer_ref"),
    "set2": ("mixture_3_sources_2", "target_reference_2", "interference_reference_2"),
}
STAGE_BINS = [4, 7, 64, 256]          # + F-1 appended per N


# ----------------------------------------------------------------------------- stand-ins
_WRITES: dict = {}


def _sf_read(path, dtype="float64", **_kw):
    fs, d = wavfile.read(path)
    if d.dtype != np.int16:
        raise ValueError(f"only int16 WAVs are expected, got {d.dtype} in {path}")
    return (d.astype(np.float64) / 32768.0).astype(dtype), fs


def _sf_write(path, data, fs, *_a, **_kw):
    _WRITES[os.path.basename(str(path))] = np.array(data, copy=True)


def install_reference():
    sf = types.ModuleType("soundfile")
    sf.read = _sf_read
    sf.write = _sf_write
    sys.modules["soundfile"] = sf
    import matplotlib
    matplotlib.use("Agg")
    for p in (REF, os.path.join(REF, "scripts"), os.path.join(REF, "Final_pipeline")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from rt_av_zoom.core import masked_mvdr, oracle_debug  # noqa: F401
    import run_metrics  # noqa: F401
    from src import metrics  # noqa: F401  (Final_pipeline/src/metrics.py)
    return oracle_debug, masked_mvdr, run_metrics, metrics


@contextlib.contextmanager
def capture():
    """Wrap scipy.signal.stft/istft and np.linalg.solve; record their I/O."""
    rec = {"stft": [], "istft": [], "solve": []}
    o_stft, o_istft, o_solve = scipy.signal.stft, scipy.signal.istft, np.linalg.solve

    def stft(*a, **k):
        r = o_stft(*a, **k)
        rec["stft"].append(r[2])
        return r

    def istft(*a, **k):
        rec["istft_in"] = np.array(a[0], copy=True)
        r = o_istft(*a, **k)
        rec["istft"].append(np.array(r[1], copy=True))  # oracle_debug normalises in place
        return r

    def solve(A, b):
        x = o_solve(A, b)
        rec["solve"].append((np.array(A), np.array(b), np.array(x)))
        return x

    scipy.signal.stft, scipy.signal.istft, np.linalg.solve = stft, istft, solve
    try:
        yield rec
    finally:
        scipy.signal.stft, scipy.signal.istft, np.linalg.solve = o_stft, o_istft, o_solve


def load_triple(name):
    mix, tgt, itf = TRIPLES[name]
    _, m = wavfile.read(os.path.join(INPUTS, mix + ".wav"))
    _, t = wavfile.read(os.path.join(INPUTS, tgt + ".wav"))
    _, i = wavfile.read(os.path.join(INPUTS, itf + ".wav"))
    return m, t, i


def run_oracle_debug(od, mix16, tgt16, int16_, n_fft, hop, sigma):
    """Run the reference oracle_debug.main() on int16 arrays; return (out, rec)."""
    with tempfile.TemporaryDirectory() as td:
        outdir = os.path.join(td, od.OUTDIR)
        os.makedirs(outdir)
        wavfile.write(os.path.join(outdir, "mixture.wav"), 16000, mix16)
        wavfile.write(os.path.join(outdir, "target_reference.wav"), 16000, tgt16)
        wavfile.write(os.path.join(outdir, "interference_reference.wav"), 16000, int16_)
        od.N_FFT, od.N_HOP, od.SIGMA = n_fft, hop, sigma
        cwd = os.getcwd()
        os.chdir(td)
        _WRITES.clear()
        try:
            with contextlib.redirect_stdout(open(os.devnull, "w")), capture() as rec:
                od.main()
        finally:
            os.chdir(cwd)
        return _WRITES["output_oracle.wav"], rec


def run_masked_mvdr(mm, mix16, n_fft, hop, sigma):
    """Run the reference heuristic masked_mvdr.main(dir); return (out, rec)."""
    with tempfile.TemporaryDirectory() as td:
        world = os.path.join(td, "run", "World_Outputs")
        os.makedirs(world)
        wavfile.write(os.path.join(world, "mixture_3_sources.wav"), 16000, mix16)
        mm.N_FFT, mm.N_HOP, mm.SIGMA = n_fft, hop, sigma
        _WRITES.clear()
        with contextlib.redirect_stdout(open(os.devnull, "w")), capture() as rec:
            mm.main(world)
        import matplotlib.pyplot as plt
        plt.close("all")
        return _WRITES["output_masked_mvdr.wav"], rec


def stage_dict(rec, n_fft):
    F = n_fft // 2 + 1
    bins = STAGE_BINS + [F - 1]
    Y = rec["stft"][0]
    out = {"bins": np.array(bins), "Y_mix": Y[:, bins, :]}
    if len(rec["stft"]) >= 3:
        out["S_tgt"] = rec["stft"][1][bins, :]
        out["S_int"] = rec["stft"][2][bins, :]
    # solve() calls happen for bins with f >= 100 Hz, in order.
    f = np.fft.rfftfreq(n_fft, 1 / 16000)
    solved = [k for k in range(F) if f[k] >= 100]
    A = np.stack([s[0] for s in rec["solve"]])
    x = np.stack([s[2][:, 0] for s in rec["solve"]])
    d = np.stack([s[1][:, 0] for s in rec["solve"]])
    sel = [solved.index(k) for k in bins if k in solved]
    out["solve_bins"] = np.array([k for k in bins if k in solved])
    out["R_loaded"] = A[sel]
    out["d"] = d[sel]
    out["w_unnorm"] = x[sel]
    out["S_final"] = rec["istft_in"][bins, :]
    return out


# ----------------------------------------------------------------------------- Final_pipeline
class _MaskFeeder:
    """Stand-in for Final_pipeline's TFLiteBeamformer: the .tflite model is absent
    (.MISSING_LARGE_BLOBS:1) and TensorFlow is not installed, so predict_mask returns
    the oracle TARGET mask of the chunk, |S_t| >= |S_i| (SURVEY 8(c) hybrid row), and
    records the features the reference computed for it."""
    masks: list = []
    features: list = []

    def __init__(self, model_path):
        self.i = 0

    def predict_mask(self, log_mag, raw_ipd):
        _MaskFeeder.features.append((np.array(log_mag), np.array(raw_ipd)))
        m = _MaskFeeder.masks[self.i]
        self.i += 1
        return m


def install_final_pipeline():
    tf = types.ModuleType("tensorflow")
    tf.lite = types.SimpleNamespace(Interpreter=None)
    sys.modules.setdefault("tensorflow", tf)
    from src import config, inference  # Final_pipeline/src (on sys.path via install_reference)
    return inference, config


def chunk_target_masks(tgt, itf, n_total, chunk=32000, hop=16000, n_fft=1024):
    """Per-chunk oracle target masks with the driver's chunking (inference.py:171-181)."""
    masks = []
    for c in range(int(np.ceil(n_total / hop))):
        seg_t = tgt[c * hop:c * hop + chunk]
        seg_i = itf[c * hop:c * hop + chunk]
        seg_t = np.pad(seg_t, (0, chunk - len(seg_t)))
        seg_i = np.pad(seg_i, (0, chunk - len(seg_i)))
        _, _, St = scipy.signal.stft(seg_t, fs=16000, nperseg=n_fft, noverlap=n_fft - n_fft // 2)
        _, _, Si = scipy.signal.stft(seg_i, fs=16000, nperseg=n_fft, noverlap=n_fft - n_fft // 2)
        masks.append((np.abs(St) >= np.abs(Si)).astype(np.float32))
    return masks


def run_enhance_audio(inference, config, mix16, tgt, itf):
    """Run Final_pipeline enhance_audio (inference.py:144-237) on a stereo int16 mixture
    with the oracle target masks; returns (final output, first hybrid call's I/O)."""
    calls = []
    orig_bf = inference.hybrid_hard_null_bf

    def bf(Y, mask, f_bins):
        S = orig_bf(Y, mask, f_bins)
        if not calls:
            calls.append((np.array(Y), np.array(mask), np.array(f_bins), np.array(S)))
        return S

    _MaskFeeder.masks = chunk_target_masks(tgt, itf, len(mix16))
    _MaskFeeder.features = []
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "mixture.wav")
        wavfile.write(inp, 16000, mix16)
        old = (config.RESULTS_DIR, inference.TFLiteBeamformer, inference.hybrid_hard_null_bf)
        config.RESULTS_DIR = td
        inference.TFLiteBeamformer = _MaskFeeder
        inference.hybrid_hard_null_bf = bf
        _WRITES.clear()
        try:
            with contextlib.redirect_stdout(open(os.devnull, "w")):
                inference.enhance_audio("golden", inp, os.path.join(td, "absent.tflite"))
        finally:
            config.RESULTS_DIR, inference.TFLiteBeamformer, inference.hybrid_hard_null_bf = old
    return _WRITES["golden_enhanced.wav"], calls[0], list(_MaskFeeder.features)


def gen_final_pipeline(trip, run_metrics, save):
    inference, config = install_final_pipeline()
    for k, (m, t, i) in trip.items():
        tf = t.astype(np.float32) / 32768.0
        itf = i.astype(np.float32) / 32768.0
        out, (Y, mask, fb, S), feats = run_enhance_audio(inference, config, m, tf, itf)
        L = min(len(out), len(tf))
        sdr_o, sir_o = run_metrics.calculate_metrics_manual(out[:L], tf[:L], itf[:L])
        arrays = dict(chunk=config.WIN_SIZE, hop=config.WIN_SIZE // 2, n_fft=config.N_FFT,
                      mic_d=config.MIC_DIST, c=config.C_SPEED, out=out.astype(np.float32),
                      sumsq=np.sum(out ** 2), sir_out=sir_o, sdr_out=sdr_o,
                      n_chunks=len(_MaskFeeder.masks))
        if k == "test":
            arrays.update(chunk0_Y=Y.astype(np.complex64), chunk0_mask=mask, chunk0_f=fb,
                          chunk0_S=S.astype(np.complex64),
                          chunk0_logmag=feats[0][0].astype(np.float32),
                          chunk0_ipd=feats[0][1].astype(np.float32))
        save(f"hybrid_{k}.npz", **arrays)


def gen_srp(trip, save):
    """scripts/debug_srp.py main() on each bundled mixture; the power map is captured
    from its plt.plot call (the script only plots it)."""
    import debug_srp  # scripts/ (on sys.path via install_reference)
    for k, (m, _, _) in trip.items():
        got = {}
        orig = debug_srp.plt.plot

        def plot(*a, **kw):
            if "x" not in got:
                got["x"], got["y"] = np.array(a[0]), np.array(a[1])
            return orig(*a, **kw)
        with tempfile.TemporaryDirectory() as td:
            world = os.path.join(td, "run", "World_Outputs")
            os.makedirs(world)
            wavfile.write(os.path.join(world, "mixture_3_sources.wav"), 16000, m)
            debug_srp.plt.plot = plot
            try:
                with contextlib.redirect_stdout(open(os.devnull, "w")):
                    debug_srp.main(world)
            finally:
                debug_srp.plt.plot = orig
                debug_srp.plt.close("all")
        save(f"srp_{k}.npz", angles=got["x"], power_db=got["y"], n_fft=512, mic_d=debug_srp.D,
             c=debug_srp.C, f_lo=200.0, f_hi=4000.0)


def run_oracle_reverb(orv, mix16, tgt16, int16_, n_fft, sigma, hp):
    """Run rt_av_zoom/core/oracle_reverb.py main(args) (:41-174) on int16 arrays. Its
    input is the WPE output mixture_wpe.wav; WPE (nara_wpe) is absent and out of scope,
    so the bundled mixture is handed over under that name. Returns (out, rec)."""
    with tempfile.TemporaryDirectory() as td:
        wavfile.write(os.path.join(td, "mixture_wpe.wav"), 16000, mix16)
        wavfile.write(os.path.join(td, "target_reference.wav"), 16000, tgt16)
        wavfile.write(os.path.join(td, "interference_reference.wav"), 16000, int16_)
        orv.N_FFT, orv.N_HOP = n_fft, n_fft // 2
        _WRITES.clear()
        args = types.SimpleNamespace(outdir=td, sigma=sigma, hp=hp)
        with contextlib.redirect_stdout(open(os.devnull, "w")), capture() as rec:
            orv.main(args)
        return _WRITES["output_oracle_reverb.wav"], rec


def gen_reverb(trip, run_metrics, save):
    from rt_av_zoom.core import oracle_reverb as orv
    cases = [(512, 1e-3, 100.0), (512, 1e-7, 200.0), (1024, 1e-3, 100.0)]
    for k, (m, t, i) in trip.items():
        tf = t.astype(np.float32) / 32768.0
        itf = i.astype(np.float32) / 32768.0
        for n, s, hp in cases:
            out, rec = run_oracle_reverb(orv, m, t, i, n, s, hp)
            L = min(len(out), len(tf))
            _, sir_o = run_metrics.calculate_metrics_manual(out[:L], tf[:L], itf[:L])
            save(f"reverb_{k}_n{n}_s{s:g}_hp{hp:g}.npz", n_fft=n, hop=n // 2, sigma=s, hp=hp,
                 out_len=len(out), out_stride16=out[::16].astype(np.float32),
                 out_head=out[:4096].astype(np.float32), sumsq=np.sum(out ** 2),
                 peak_raw=np.max(np.abs(rec["istft"][0])), sir_out=sir_o)
    seg = slice(40000, 64000)
    m, t, i = trip["test"]
    out, rec = run_oracle_reverb(orv, m[seg], t[seg], i[seg], 512, 1e-3, 100.0)
    save("reverb_excerpt_test_n512.npz", seg=np.array([seg.start, seg.stop]), n_fft=512,
         sigma=1e-3, hp=100.0, out=out.astype(np.float32),
         S_final=rec["istft_in"].astype(np.complex128))


UNET_SEED = 20250101


def unet_checksum(state_dict):
    """(count, sum |p|, sum p * index-weight) of a state_dict in fp64: pins the weights."""
    n, s1, s2 = 0, 0.0, 0.0
    for k in sorted(state_dict):
        v = state_dict[k].detach().double().flatten().numpy()
        n += v.size
        s1 += float(np.abs(v).sum())
        s2 += float((v * np.linspace(1.0, 2.0, v.size)).sum())
    return np.array([n, s1, s2])


def gen_neural(trip, run_metrics, save):
    """full_audio_generating_pipeline/inference.py main_deploy (:120-167) + process_chunk
    (:88-118). The trained weights mask_3.pth are absent upstream (.MISSING_LARGE_BLOBS:2),
    so the reference's own FreqPreservingUNet (:29-67) is built with random init under
    torch.manual_seed(UNET_SEED), eval mode, and saved as mask_3.pth for main_deploy to
    load. mir_eval (imported at :10, used only by code main_deploy does not call) is
    absent: an empty stand-in module is injected. The module reads config.json from the
    working directory at import (:15-16); the reference's own config.json is copied there."""
    import importlib

    import torch
    me = types.ModuleType("mir_eval")
    me.separation = types.SimpleNamespace(bss_eval_sources=None)
    sys.modules.setdefault("mir_eval", me)
    sys.modules.setdefault("mir_eval.separation", me.separation)
    pipe = os.path.join(REF, "rt_av_zoom", "core", "full_audio_generating_pipeline")
    with tempfile.TemporaryDirectory() as td:
        shutil.copy(os.path.join(pipe, "config.json"), td)
        cwd = os.getcwd()
        os.chdir(td)
        try:
            inf = importlib.import_module("rt_av_zoom.core.full_audio_generating_pipeline.inference")
            torch.manual_seed(UNET_SEED)
            model = inf.FreqPreservingUNet()
            sd = model.state_dict()
            torch.save(sd, "mask_3.pth")
            conf = json.load(open("config.json"))
            rec = {"X": [], "M": []}
            orig_fwd = inf.FreqPreservingUNet.forward

            def fwd(self, x):
                m = orig_fwd(self, x)
                rec["X"].append(x.detach().numpy().copy())
                rec["M"].append(m.detach().numpy().copy())
                return m

            def deploy(mix16):
                wavfile.write("input.wav", 16000, mix16)
                rec["X"].clear()
                rec["M"].clear()
                _WRITES.clear()
                inf.FreqPreservingUNet.forward = fwd
                try:
                    with contextlib.redirect_stdout(open(os.devnull, "w")):
                        inf.main_deploy("input.wav")
                finally:
                    inf.FreqPreservingUNet.forward = orig_fwd
                return _WRITES["enhanced_input.wav"]

            common = dict(seed=UNET_SEED, checksum=unet_checksum(sd),
                          keys=np.array(sorted(sd)), n_fft=conf["n_fft"], hop=conf["hop_len"],
                          mic_d=conf["d"], chunk=conf["train_seg_samples"], sigma=inf.SIGMA)
            for k, (m, t, i) in trip.items():
                out = deploy(m)
                tf = t.astype(np.float32) / 32768.0
                itf = i.astype(np.float32) / 32768.0
                L = min(len(out), len(tf))
                _, sir_o = run_metrics.calculate_metrics_manual(out[:L], tf[:L], itf[:L])
                save(f"neural_{k}.npz", **common, out_len=len(out),
                     out_stride16=out[::16].astype(np.float32), out_head=out[:4096].astype(np.float32),
                     sumsq=np.sum(out ** 2), sir_out=sir_o, n_chunks=len(rec["M"]))
            seg = slice(40000, 88000)
            m, _, _ = trip["test"]
            out = deploy(m[seg])
            save("neural_excerpt_test.npz", **common, seg=np.array([seg.start, seg.stop]),
                 out=out.astype(np.float32), masks=np.concatenate(rec["M"]).astype(np.float32),
                 feat0=rec["X"][0][0].astype(np.float32))
        finally:
            os.chdir(cwd)


def gen_world(trip, save):
    """full_audio_generating_pipeline/world_building.py mix_and_save (:68-100) on three
    1.5-s mono excerpts of the bundled references (target first). kagglehub and librosa
    are imported at module level but not used on this path (the WAVs are already 16 kHz,
    so load_resample never resamples): empty stand-ins are injected."""
    import importlib
    for name in ("kagglehub", "librosa"):
        sys.modules.setdefault(name, types.ModuleType(name))
    wb = importlib.import_module("rt_av_zoom.core.full_audio_generating_pipeline.world_building")
    seg = slice(40000, 48000)
    srcs = [trip["test"][1][seg], trip["test"][2][seg], trip["set2"][1][seg]]
    with tempfile.TemporaryDirectory() as td:
        files = []
        for j, s in enumerate(srcs):
            files.append(os.path.join(td, f"src{j}.wav"))
            wavfile.write(files[-1], 16000, s)
        cwd = os.getcwd()
        os.chdir(td)
        _WRITES.clear()
        try:
            with contextlib.redirect_stdout(open(os.devnull, "w")):
                wb.mix_and_save(files, "golden")
        finally:
            os.chdir(cwd)
    save("world_mix.npz", sources=np.stack(srcs), d=wb.D,
         angles=np.array([wb.ANGLE_TARGET, wb.ANGLE_INTERFERER_A, wb.ANGLE_INTERFERER_B]),
         mixture=_WRITES["mixture_golden.wav"], target_ref=_WRITES["target_ref_golden.wav"],
         interf_ref=_WRITES["interf_ref_golden.wav"])


def gen_report(trip, metrics, save):
    """Final_pipeline/src/metrics.py evaluate_run on a simulated-run folder built from the
    test triple (stereo target/interference/mixture as simulation.py:205-211 writes them)
    and the int16-quantised hybrid golden output as <run>_enhanced.wav."""
    from src import config
    m, t, i = trip["test"]
    out = np.load(os.path.join(HERE, "hybrid_test.npz"))["out"]
    est16 = np.clip(np.round(out.astype(np.float64) * 32768), -32768, 32767).astype(np.int16)
    with tempfile.TemporaryDirectory() as td:
        sim = os.path.join(td, "simulated", "golden_run")
        res = os.path.join(td, "results", "golden_run_results")
        os.makedirs(sim)
        os.makedirs(res)
        wavfile.write(os.path.join(sim, "mixture.wav"), 16000, m)
        wavfile.write(os.path.join(sim, "target.wav"), 16000, np.stack([t, t], 1))
        wavfile.write(os.path.join(sim, "interference.wav"), 16000, np.stack([i, i], 1))
        wavfile.write(os.path.join(res, "golden_run_enhanced.wav"), 16000, est16)
        old = (config.SIM_DIR, config.RESULTS_DIR)
        config.SIM_DIR, config.RESULTS_DIR = os.path.join(td, "simulated"), os.path.join(td, "results")
        try:
            with contextlib.redirect_stdout(open(os.devnull, "w")):
                metrics.evaluate_run("golden_run")
        finally:
            config.SIM_DIR, config.RESULTS_DIR = old
        report = open(os.path.join(res, "report.txt")).read()
        csv_text = open(os.path.join(td, "results", "batch_metrics.csv")).read()
    save("report_test.npz", est16=est16, report=np.array(report), csv=np.array(csv_text))


def gen_spectral(trip, save):
    """The spectral-domain operators on STFTs of 2-s chunks of the bundled mixtures:
    rt_av_zoom/core/tf_lite_version/inference.py batch_mvdr (:85-179) with the module's
    own get_all_steering_vectors (:53-81) and SIGMA (:46), and its chunk driver's
    post-filter + istft (:347-352). The module imports tensorflow at top level (absent;
    unused by these functions): an empty stand-in is injected; its config.json is the
    reference's own (read from the module directory). Masks are float32 like a TFLite
    output: the chunk's oracle target mask (|S_t| >= |S_i|) and a soft one
    (sigmoid(log|S_t| - log|S_i|)). One case zeroes bin 0 of Y at sigma = 0 so the single
    np.linalg.solve raises LinAlgError and every bin takes the fallback (:149-153)."""
    import importlib
    tf = types.ModuleType("tensorflow")
    tf.lite = types.SimpleNamespace(Interpreter=None)
    sys.modules.setdefault("tensorflow", tf)
    tl_dir = os.path.join(REF, "rt_av_zoom", "core", "tf_lite_version")
    cwd = os.getcwd()
    os.chdir(tl_dir)  # its config.json (read-only use)
    try:
        with contextlib.redirect_stdout(open(os.devnull, "w")):
            tl = importlib.import_module("rt_av_zoom.core.tf_lite_version.inference")
    finally:
        os.chdir(cwd)
    n_fft, hop, fs = tl.N_FFT, tl.HOP, tl.FS
    cases = [("test_ibm", "test", 0, "ibm", tl.SIGMA), ("test_soft", "test", 0, "soft", tl.SIGMA),
             ("set2_soft", "set2", 16000, "soft", tl.SIGMA),
             ("test_singular", "test", 32000, "soft", 0.0)]
    for name, k, start, kind, sigma in cases:
        m, t, i = trip[k]
        seg = slice(start, start + 32000)
        chunk = (m[seg].astype(np.float64) / 32768.0).astype(np.float32)
        f_bins, _, Y = scipy.signal.stft(chunk.T, fs=fs, nperseg=n_fft, noverlap=n_fft - hop)
        st_ = (t[seg].astype(np.float64) / 32768.0).astype(np.float32)
        si_ = (i[seg].astype(np.float64) / 32768.0).astype(np.float32)
        _, _, St = scipy.signal.stft(st_, fs=fs, nperseg=n_fft, noverlap=n_fft - hop)
        _, _, Si = scipy.signal.stft(si_, fs=fs, nperseg=n_fft, noverlap=n_fft - hop)
        if kind == "ibm":
            mask = (np.abs(St) >= np.abs(Si)).astype(np.float32)
        else:
            z = np.log(np.abs(St) + 1e-7) - np.log(np.abs(Si) + 1e-7)
            mask = (1.0 / (1.0 + np.exp(-z))).astype(np.float32)
        if name == "test_singular":
            Y = Y.copy()
            Y[:, 0, :] = 0
        d_vecs = tl.get_all_steering_vectors(f_bins, tl.ANGLE_TARGET, tl.D, tl.C)
        raised = []
        o_solve = np.linalg.solve

        def solve(A, b):  # records whether the reference's single solve raised
            try:
                return o_solve(A, b)
            except np.linalg.LinAlgError:
                raised.append(True)
                raise
        np.linalg.solve = solve
        try:
            S_out = tl.batch_mvdr(Y, mask, f_bins, d_vecs, sigma)
        finally:
            np.linalg.solve = o_solve
        S_final = S_out * np.maximum(mask, 0.05)
        _, chunk_out = scipy.signal.istft(S_final, fs=fs, nperseg=n_fft, noverlap=n_fft - hop)
        save(f"spectral_{name}.npz", n_fft=n_fft, hop=hop, fs=fs, sigma=sigma, d=tl.D, c=tl.C,
             angle=tl.ANGLE_TARGET, Y=Y.astype(np.complex64), mask=mask, f_bins=f_bins,
             d_vectors=d_vecs[:, :, 0], S_out=S_out.astype(np.complex64),
             chunk_out=chunk_out.astype(np.float32), fallback=bool(raised))


class _TLMaskFeeder:
    """Stand-in for tf_lite_version's TFLiteBeamformer (inference.py:185-239): the
    .tflite model is absent and TensorFlow is not installed, so predict_mask(log_mag, ipd)
    returns the next chunk's precomputed target mask and records the features the
    reference computed for it (:296-300)."""
    masks: list = []
    features: list = []

    def __init__(self, model_path="mask_estimator.tflite"):
        self.i = 0

    def predict_mask(self, log_mag, ipd):
        _TLMaskFeeder.features.append((np.array(log_mag), np.array(ipd)))
        m = _TLMaskFeeder.masks[self.i]
        self.i += 1
        return m


def chunk_soft_masks(tgt, itf, n_total, chunk=32000, hop=16000, n_fft=1024):
    """Per-chunk soft target masks sigmoid(log|S_t| - log|S_i|) (float32, like a TFLite
    output) with process_audio_file's chunking (inference.py:269-289)."""
    masks = []
    for c in range(int(np.ceil(n_total / hop))):
        seg_t = np.pad(tgt[c * hop:c * hop + chunk], (0, max(0, chunk - len(tgt[c * hop:c * hop + chunk]))))
        seg_i = np.pad(itf[c * hop:c * hop + chunk], (0, max(0, chunk - len(itf[c * hop:c * hop + chunk]))))
        _, _, St = scipy.signal.stft(seg_t, fs=16000, nperseg=n_fft, noverlap=n_fft - n_fft // 2)
        _, _, Si = scipy.signal.stft(seg_i, fs=16000, nperseg=n_fft, noverlap=n_fft - n_fft // 2)
        z = np.log(np.abs(St) + 1e-7) - np.log(np.abs(Si) + 1e-7)
        masks.append((1.0 / (1.0 + np.exp(-z))).astype(np.float32))
    return masks


def gen_tflite(trip, run_metrics, save):
    """rt_av_zoom/core/tf_lite_version/inference.py process_audio_file (:245-391) run on
    each bundled stereo mixture, its model replaced by _TLMaskFeeder (soft target masks of
    the chunk's references); the module reads its own config.json at import (d = 0.04)."""
    import importlib
    tf = types.ModuleType("tensorflow")
    tf.lite = types.SimpleNamespace(Interpreter=None)
    sys.modules.setdefault("tensorflow", tf)
    tl_dir = os.path.join(REF, "rt_av_zoom", "core", "tf_lite_version")
    cwd = os.getcwd()
    os.chdir(tl_dir)  # its config.json (read-only use)
    try:
        with contextlib.redirect_stdout(open(os.devnull, "w")):
            tl = importlib.import_module("rt_av_zoom.core.tf_lite_version.inference")
    finally:
        os.chdir(cwd)
    for k, (m, t, i) in trip.items():
        tf32 = t.astype(np.float32) / 32768.0
        if32 = i.astype(np.float32) / 32768.0
        _TLMaskFeeder.masks = chunk_soft_masks(tf32, if32, len(m), chunk=tl.WIN_SIZE,
                                               hop=tl.WIN_SIZE // 2, n_fft=tl.N_FFT)
        _TLMaskFeeder.features = []
        old = tl.TFLiteBeamformer
        tl.TFLiteBeamformer = _TLMaskFeeder
        with tempfile.TemporaryDirectory() as td:
            inp = os.path.join(td, "mixture.wav")
            wavfile.write(inp, 16000, m)
            model = os.path.join(td, "absent.tflite")
            open(model, "wb").close()  # the size print needs a file; the feeder needs none
            _WRITES.clear()
            try:
                with contextlib.redirect_stdout(open(os.devnull, "w")):
                    tl.process_audio_file(inp, os.path.join(td, "enhanced.wav"), model)
            finally:
                tl.TFLiteBeamformer = old
        out = _WRITES["enhanced.wav"]
        L = min(len(out), len(tf32))
        sdr_o, sir_o = run_metrics.calculate_metrics_manual(out[:L], tf32[:L], if32[:L])
        lm, ipd = _TLMaskFeeder.features[0]
        save(f"tflite_{k}.npz", chunk=tl.WIN_SIZE, n_fft=tl.N_FFT, hop=tl.HOP, d=tl.D, c=tl.C,
             sigma=tl.SIGMA, masks=np.stack(_TLMaskFeeder.masks), out=out.astype(np.float32),
             out_len=len(out), sumsq=np.sum(out ** 2), sir_out=sir_o, sdr_out=sdr_o,
             chunk0_logmag=lm.astype(np.float32), chunk0_ipd=ipd.astype(np.float32))


def main():
    od, mm, run_metrics, metrics = install_reference()
    mpath = os.path.join(HERE, "MANIFEST.json")
    manifest = {"generator": "tests/golden/make_golden.py", "reference": REF,
                "scipy": scipy.__version__, "numpy": np.__version__, "files": {}}
    only = sys.argv[1:]  # e.g. "hybrid": regenerate one family, keep the rest
    if only and os.path.exists(mpath):
        manifest["files"] = json.load(open(mpath))["files"]

    def save(name, **arrays):
        path = os.path.join(HERE, name)
        np.savez_compressed(path, **arrays)
        manifest["files"][name] = sorted(arrays)
        print("wrote", name, os.path.getsize(path) // 1024, "KiB")

    trip = {k: load_triple(k) for k in TRIPLES}
    if only:
        if "hybrid" in only:
            gen_final_pipeline(trip, run_metrics, save)
        if "srp" in only:
            gen_srp(trip, save)
        if "report" in only:
            gen_report(trip, metrics, save)
        if "reverb" in only:
            gen_reverb(trip, run_metrics, save)
        if "neural" in only:
            gen_neural(trip, run_metrics, save)
        if "world" in only:
            gen_world(trip, save)
        if "spectral" in only:
            gen_spectral(trip, save)
        if "tflite" in only:
            gen_tflite(trip, run_metrics, save)
        with open(mpath, "w") as fh:
            json.dump(manifest, fh, indent=1, sort_keys=True)
        return

    # -- bundled inputs (data files of the reference, int16) --------------------
    for k, (m, t, i) in trip.items():
        save(f"inputs_{k}.npz", mix=m, tgt=t, int=i)

    # -- full-length oracle_debug runs ------------------------------------------
    full_cases = [(k, n, s) for k in TRIPLES for n in (512, 1024) for s in (1.0, 1e-5, 1e-7)]
    for k, n, s in full_cases:
        m, t, i = trip[k]
        out, rec = run_oracle_debug(od, m, t, i, n, n // 2, s)
        raw = rec["istft"][0]
        tf = t.astype(np.float32) / 32768.0
        itf = i.astype(np.float32) / 32768.0
        L = min(len(out), len(tf))
        sdr_o, sir_o = run_metrics.calculate_metrics_manual(out[:L], tf[:L], itf[:L])
        mix0 = m[:, 0].astype(np.float32) / 32768.0
        sdr_i, sir_i = run_metrics.calculate_metrics_manual(mix0[:L], tf[:L], itf[:L])
        osinr, osir = metrics.calculate_osnr_osir(out[:L].astype(np.float64),
                                                  tf[:L].astype(np.float64),
                                                  itf[:L].astype(np.float64))
        save(f"full_{k}_n{n}_s{s:g}.npz", n_fft=n, hop=n // 2, sigma=s,
             out_len=len(out), out_stride16=out[::16].astype(np.float32),
             out_head=out[:4096].astype(np.float32), sumsq=np.sum(out ** 2),
             peak_raw=np.max(np.abs(raw)), sir_in=sir_i, sdr_in=sdr_i, sir_out=sir_o,
             sdr_out=sdr_o, osinr_out=osinr, osir_out=osir)

    # -- 1.5-s excerpts (inputs = inputs_<k>.npz[seg]): full outputs + stage intermediates ----------------------
    seg = slice(40000, 64000)
    for k in TRIPLES:
        m, t, i = trip[k]
        m, t, i = m[seg], t[seg], i[seg]
        for n in (512, 1024):
            for s in (1.0, 1e-7):
                out, rec = run_oracle_debug(od, m, t, i, n, n // 2, s)
                arrays = dict(seg=np.array([seg.start, seg.stop]), n_fft=n, hop=n // 2, sigma=s,
                              out=out.astype(np.float32), peak_raw=np.max(np.abs(rec["istft"][0])))
                if k == "test":
                    for key, v in stage_dict(rec, n).items():
                        arrays["stage_" + key] = v
                save(f"excerpt_{k}_n{n}_s{s:g}.npz", **arrays)

    # -- heuristic IPD path (masked_mvdr.main) -----------------------------------
    for k in TRIPLES:
        m, t, i = trip[k]
        for n in (512, 1024):
            out, rec = run_masked_mvdr(mm, m, n, n // 2, 1e-7)
            tf = t.astype(np.float32) / 32768.0
            itf = i.astype(np.float32) / 32768.0
            L = min(len(out), len(tf))
            _, sir_o = run_metrics.calculate_metrics_manual(out[:L], tf[:L], itf[:L])
            Y = rec["stft"][0]
            ipd_mask = mm.compute_hard_geometric_mask(Y, None)
            save(f"ipd_{k}_n{n}.npz", n_fft=n, hop=n // 2, sigma=1e-7, out_len=len(out),
                 out_stride16=out[::16].astype(np.float32), out_head=out[:4096].astype(np.float32),
                 sumsq=np.sum(out ** 2), sir_out=sir_o,
                 mask_low_count=np.sum(ipd_mask < 1.0), mask_low_bins=np.nonzero(
                     (ipd_mask < 1.0).any(axis=1))[0])
        # excerpt with full output
        mseg = m[seg]
        for n in (512, 1024):
            out, _ = run_masked_mvdr(mm, mseg, n, n // 2, 1e-7)
            save(f"ipd_excerpt_{k}_n{n}.npz", seg=np.array([seg.start, seg.stop]), n_fft=n,
                 hop=n // 2, sigma=1e-7, out=out.astype(np.float32))

    # -- metric functions on fixed vectors ---------------------------------------
    rng = np.random.default_rng(7)
    o, t, i = rng.standard_normal((3, 5000))
    o = 0.7 * t + 0.2 * i + 0.1 * o
    sdr, sir = run_metrics.calculate_metrics_manual(o, t, i)
    osinr, osir = metrics.calculate_osnr_osir(o, t, i)
    save("metrics_vectors.npz", o=o, t=t, i=i, sdr=sdr, sir=sir, osinr=osinr, osir=osir)

    # -- steering vectors --------------------------------------------------------
    f = np.fft.rfftfreq(1024, 1 / 16000)
    sv = np.stack([mm.get_steering_vector(a, fk, d, 343.0)[:, 0]
                   for a, d in ((90.0, 0.01), (40.0, 0.08), (130.0, 0.04)) for fk in f])
    save("steering.npz", f=f, sv=sv.reshape(3, len(f), 2))

    # -- Final_pipeline hybrid hard-null driver (run.py inf / batch_run) -----------
    gen_final_pipeline(trip, run_metrics, save)
    gen_srp(trip, save)
    gen_report(trip, metrics, save)
    gen_reverb(trip, run_metrics, save)
    gen_neural(trip, run_metrics, save)
    gen_world(trip, save)
    gen_spectral(trip, save)
    gen_tflite(trip, run_metrics, save)

    with open(os.path.join(HERE, "MANIFEST.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
