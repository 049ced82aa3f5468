"""GPU tests of the reference-surface mirrors (oracle_debug.main, masked_mvdr.main,
batch_run.run_batch) end to end through the C ABI, against the goldens / oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import golden, triple_f32
from oracle import avz_oracle as O

pytestmark = pytest.mark.gpu


def _write_triple(d, name, mix_name="mixture.wav", tgt_name="target_reference.wav",
                  int_name="interference_reference.wav"):
    from avz import wavio
    g = golden(f"inputs_{name}.npz")
    os.makedirs(d, exist_ok=True)
    wavio.write(os.path.join(d, mix_name), g["mix"] / 32768.0, 16000)
    if tgt_name:
        wavio.write(os.path.join(d, tgt_name), g["tgt"] / 32768.0, 16000)
        wavio.write(os.path.join(d, int_name), g["int"] / 32768.0, 16000)


def test_oracle_debug_main_mirror(gpu_device, tmp_path):
    from avz import oracle_debug
    outdir = str(tmp_path / oracle_debug.OUTDIR)
    _write_triple(outdir, "test")
    s_out = oracle_debug.main(outdir)          # shipped settings: 512/256, sigma 1
    g = golden("full_test_n512_s1.npz")
    assert len(s_out) == int(g["out_len"])
    assert np.max(np.abs(s_out[::16] - g["out_stride16"])) <= 1e-4
    assert os.path.exists(os.path.join(outdir, "output_oracle.wav"))
    _, tgt, itf = triple_f32("test")
    L = len(tgt)
    assert abs(O.projection_sdr_sir(s_out[:L].astype(np.float64), tgt, itf)[1]
               - float(g["sir_out"])) <= 0.01


def test_masked_mvdr_main_mirror(gpu_device, tmp_path):
    from avz import masked_mvdr
    world = str(tmp_path / "run" / "World_Outputs")
    _write_triple(world, "set2", mix_name="mixture_3_sources.wav", tgt_name=None)
    s_out = masked_mvdr.main(world)
    g = golden("ipd_set2_n512.npz")
    assert len(s_out) == int(g["out_len"])
    assert np.max(np.abs(s_out[::16] - g["out_stride16"])) <= 1e-4
    assert os.path.exists(str(tmp_path / "run" / "MVDR_Outputs" / "output_masked_mvdr.wav"))


def test_ipd_mask_helper_matches_reference_semantics(gpu_device):
    from avz import masked_mvdr
    mix, _, _ = triple_f32("test", (0, 20000))
    _, _, Y = O.stft(mix, nperseg=512, noverlap=256)
    m = masked_mvdr.compute_hard_geometric_mask(Y).cpu().numpy()
    np.testing.assert_array_equal(m, O.ipd_mask_noise(Y))


def test_device_metrics_match_host(gpu_device):
    """avz_projection_metrics (float32 signals, fp64 inner products) against the
    reference formulas on the same float32 values (the reference reads float32 WAVs and
    computes in float64, metrics.py:91-98)."""
    from avz import metrics
    g = golden("metrics_vectors.npz")
    o, t, i = (g[k].astype(np.float32) for k in ("o", "t", "i"))
    d = lambda a: torch.from_numpy(a)[None].to(gpu_device)  # noqa: E731
    m = metrics.projection_metrics(d(o), d(t), d(i)).cpu().numpy()[0]
    f = lambda a: a.astype(np.float64)  # noqa: E731
    osinr, osir = O.osinr_osir(f(o), f(t), f(i))
    sdr, sir = O.projection_sdr_sir(f(o), f(t), f(i))
    np.testing.assert_allclose(m, [osinr, osir, sdr, sir], rtol=0, atol=1e-9)
    # float32 rounding of the inputs moves the reference's own numbers by far less than
    # the report's 0.01 dB resolution
    assert abs(m[3] - float(g["sir"])) < 1e-4


def test_device_metrics_ragged_batch(gpu_device):
    from avz import metrics
    rng = np.random.default_rng(3)
    B, S = 5, 70001
    o, t, i = (rng.standard_normal((B, S)).astype(np.float32) for _ in range(3))
    o = o + 2.0 * t
    L = [70001, 1, 4096, 33333, 12]
    d = lambda a: torch.from_numpy(a).to(gpu_device)  # noqa: E731
    m = metrics.projection_metrics(d(o), d(t), d(i), lengths=L).cpu().numpy()
    for b in range(B):
        f = lambda a: a[b, :L[b]].astype(np.float64)  # noqa: E731
        ref = list(O.osinr_osir(f(o), f(t), f(i))) + list(O.projection_sdr_sir(f(o), f(t), f(i)))
        np.testing.assert_allclose(m[b], ref, rtol=1e-9, atol=1e-9)


def test_evaluate_run_report_matches_reference(gpu_device, tmp_path):
    """metrics.evaluate_run mirror vs the report.txt / batch_metrics.csv the reference's
    Final_pipeline/src/metrics.py wrote for the same files (Date line excluded)."""
    from avz import metrics, wavio
    g = golden("report_test.npz")
    inp = golden("inputs_test.npz")
    sim = tmp_path / "simulated" / "golden_run"
    res = tmp_path / "results" / "golden_run_results"
    sim.mkdir(parents=True)
    res.mkdir(parents=True)
    f = lambda a: a.astype(np.float64) / 32768.0  # noqa: E731
    wavio.write(str(sim / "mixture.wav"), f(inp["mix"]), 16000)
    wavio.write(str(sim / "target.wav"), np.stack([f(inp["tgt"])] * 2, 1), 16000)
    wavio.write(str(sim / "interference.wav"), np.stack([f(inp["int"])] * 2, 1), 16000)
    wavio.write(str(res / "golden_run_enhanced.wav"), f(g["est16"]), 16000)
    metrics.evaluate_run("golden_run", sim_dir_root=str(tmp_path / "simulated"),
                         results_dir=str(tmp_path / "results"))
    got = (res / "report.txt").read_text().splitlines()
    ref = str(g["report"]).splitlines()
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        if not a.startswith("Date:"):
            assert a == b
    assert (tmp_path / "results" / "batch_metrics.csv").read_text() == str(g["csv"])


def test_batch_run_gpu_matches_oracle_enhancer(gpu_device):
    from avz import batch_run

    def oracle_enhance(mix, tgt, itf):
        outs = [O.oracle_debug_vec(m.cpu().numpy(), t.cpu().numpy(), i.cpu().numpy(),
                                   n_fft=1024, hop=512, sigma=1.0)
                for m, t, i in zip(mix, tgt, itf)]
        return torch.from_numpy(np.stack(outs)).to(mix.device)

    gpu = batch_run.run_batch(6, start_idx=11, seconds=1.0, batch=4, device=gpu_device)
    ref = batch_run.run_batch(6, start_idx=11, seconds=1.0, batch=4, device=gpu_device,
                              enhance=oracle_enhance)
    assert gpu.sums[4] == 6
    np.testing.assert_allclose(gpu.sums[:4] / 6, ref.sums[:4] / 6, atol=0.01)  # mean dB


def test_plan_timing_modes(gpu_device):
    """avz_plan_set_timing: mode 1 times all four kernels, mode 2 the analysis kernel
    only (NaN for the rest), 0 turns it off (get_timing then reports an argument error).
    With peak normalisation at N = 1024 the per-utterance synthesis kernel folds finalize
    (and, for plain MVDR plans, the solve) in, which then count 0 -- unless, as for this
    batch of 4 (below the CU count), it splits the utterances into step pieces, which solve
    their bins in-block and launch a piece finalize; a batch just above the CU count splits
    its partial round into pieces that finalize in-kernel (no solve, no finalize launch);
    without peak normalisation (normalize="none") all four kernels run and are timed."""
    import math

    import avz
    from avz._lib import AvzError
    from avz import synth
    mix, tgt, itf = synth.make_batch(4, n_samples=32000)
    d = [torch.from_numpy(x).to(gpu_device) for x in (mix, tgt, itf)]
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        max_batch=4, max_samples=32000)
    for mode in ("all", "analysis"):
        plan.set_timing(True, analysis_only=(mode == "analysis"))
        for _ in range(3):
            plan.run(d[0], ref_tgt=d[1], ref_int=d[2])
        t = plan.timing()
        assert t["calls"] == 3 and t["analysis"] > 0
        others = [t[k] for k in ("solve", "synthesis", "finalize")]
        if mode == "all":  # B = 4 < #CU: split into pieces, whose finalize launch runs
            assert others[0] == 0 and others[1] > 0 and others[2] > 0
        else:
            assert all(math.isnan(v) for v in others)
    R = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    mix2, tgt2, itf2 = synth.make_batch(R + 4, n_samples=32000)
    d2 = [torch.from_numpy(x).to(gpu_device) for x in (mix2, tgt2, itf2)]
    plan_i = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                          max_batch=R + 4, max_samples=32000)
    plan_i.set_timing(True)
    for _ in range(2):
        plan_i.run(d2[0], ref_tgt=d2[1], ref_int=d2[2])
    t = plan_i.timing()  # B = #CU + 4: the pieces finalize inside the synthesis launch
    assert t["calls"] == 2 and t["analysis"] > 0 and t["synthesis"] > 0
    assert t["solve"] == 0 and t["finalize"] == 0
    plan_n = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                          normalize="none", max_batch=4, max_samples=32000)
    plan_n.set_timing(True)
    for _ in range(2):
        plan_n.run(d[0], ref_tgt=d[1], ref_int=d[2])
    t = plan_n.timing()
    assert t["calls"] == 2 and all(t[k] > 0 for k in plan_n.KERNELS)
    plan.set_timing(True, analysis_only=True, period=4)  # sampled: calls 0, 4, 8
    for _ in range(9):
        plan.run(d[0], ref_tgt=d[1], ref_int=d[2])
    t = plan.timing()
    assert t["calls"] == 3 and t["analysis"] > 0
    plan.set_timing(False)
    with pytest.raises(AvzError):
        plan.timing()


def test_batch_run_gpu_all_zero_utterance_n_ok(gpu_device):
    """The HIP engine on a batch with one all-zero input: its output and peak are 0, so its
    deferred-normalised metrics are 0/0 (NaN). n_ok = B - 1, the sums are finite and equal
    the other utterances' (SURVEY 8(e)'s non-finite guard)."""
    from avz import batch_run
    B = 5
    base = batch_run.gpu_enhancer(max_batch=B, max_samples=16000)

    def enh(mix, tgt, itf):
        mix = mix.clone()
        mix[2] = 0.0
        return base(mix, tgt, itf)

    res = batch_run.run_batch(B, start_idx=20, seconds=1.0, batch=B, device=gpu_device,
                              enhance=enh)
    full = batch_run.run_batch(B, start_idx=20, seconds=1.0, batch=B, device=gpu_device)
    assert res.sums[4] == B - 1 and res.sums[5] == B and full.sums[4] == B
    assert np.all(np.isfinite(res.sums))
    assert res.rows[2]["SIR_Enh"] == "nan"
    keep = [0, 1, 3, 4]
    sir_b = sum(float(full.rows[j]["SIR_Base"]) for j in keep)
    sir_e = sum(float(full.rows[j]["SIR_Enh"]) for j in keep)
    np.testing.assert_allclose(res.sums[:2], [sir_b, sir_e], atol=0.05)
