"""Headline benchmark: beamformed TF-bins/s of the MVDR hot path on MI355X.

Default workload (BASELINE.json configs[1], the one the metric is quoted on): per GPU a
batch of B = 256 synthetic 2-mic utterances of 4.0 s (64000 samples @ 16 kHz),
2 interferers, oracle IBM mask, 1024-pt STFT / hop 512 -> F x T = 513 x 126 = 64,638
TF-bins per utterance. One step = one avz_mvdr_batch call over the whole batch: the
analysis (STFT -> IBM -> masked covariance partials), solve (fp64 MVDR), synthesis
(STFT -> apply + IBM post-filter -> iSTFT/OLA) and finalize (chunk seams, peak
normalisation) kernels, inputs resident in HBM. The timed steps alternate between two
distinct batches (2 x 262 MB of input, more than the 256 MB Infinity Cache), so no step
re-reads the previous step's input from the die. Per-kernel times come from HIP events the
plan records around each launch on the launch stream (avz_plan_set_timing).
Multi-GPU: one process per GPU, utterances sharded (weak scaling, no data-path
collective); the only collectives are the final RCCL all-reduce of the SIR metric sums
and the max-over-ranks step time. With --gpus N > 1 the per-GPU shard defaults to
configs[2]'s (B = 4096 over 8 GPUs = 512 utterances per GPU, 3 interferers).

The N = 1 default run also measures, in the same JSON line (`secondary`), every other
single-GPU configuration the same way: configs[2]'s per-GPU shard, configs[3] (IPD,
B = 1024), oracle_debug's 512/256 STFT, the batch driver's deferred normalisation and
configs[4]'s MVDR chain (4096 two-second external-mask items).

Other workloads (parity configs, measured on request, same JSON line):
  --workload ipd   configs[3]: heuristic IPD mask (masked_mvdr.py), B = 1024, no
                   post-filter, sigma 1e-7, s /= max|s| + 1e-6
  --workload unet  configs[4]: 2-s chunks of B = 1024 utterances (4096 items) ->
                   device features -> FreqPreservingUNet (PyTorch-ROCm fp32, random
                   init: weights absent upstream) -> external-mask MVDR chain ->
                   chunk overlap-add (main_deploy); value counts chunk TF-bins
                   (4096 x 513 x 64) end to end, U-Net included; the U-Net and the
                   MVDR chain are also timed alone

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "real-time-audio-visual-zooming_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
FS, SECONDS = 16000, 4.0
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, FP32 vector / matrix peak (spec)
DEFAULT_BATCH = {"ibm": 256, "ipd": 1024, "unet": 1024}
CPU_SHARE = 16  # host cores per GPU on the MI355X boxes (their CPU share; nproc shows the machine)
WORKLOAD_TEXT = {
    "ibm": "configs[1]: B={B} utterances/GPU, {k} interferers, oracle IBM, {n}-pt STFT hop {h} "
           "@16 kHz, 4.0 s utterances",
    "ipd": "configs[3]: B={B} utterances/GPU, heuristic IPD mask (masked_mvdr.py), {k} "
           "interferers, {n}-pt STFT hop {h} @16 kHz, 4.0 s utterances",
    "unet": "configs[4]: B={B} utterances/GPU -> 2-s chunks, U-Net mask (PyTorch-ROCm {unet_dtype}, "
            "random init) -> external-mask MVDR, {n}-pt STFT hop {h}, chunk OLA",
    "chain4": "configs[4] MVDR chain only: B={B} utterances/GPU -> 2-s chunk items, external "
              "target mask (a fixed synthetic mask stands in for the U-Net output) -> MVDR, "
              "max(M, 0.05) post-filter, iSTFT, {n}-pt STFT hop {h}",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(DEFAULT_BATCH), default="ibm")
    ap.add_argument("--batch", type=int, default=0,
                    help="utterances per GPU (0: workload default; ibm at N > 1: 512, configs[2])")
    ap.add_argument("--interferers", type=int, default=0,
                    help="interferers per scene (0: 2; ibm at N > 1: 3, configs[2])")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="time box of the CPU baseline workers")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help=f"0: min({CPU_SHARE}, available cores) -- the box's CPU share per GPU")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="N = 1: skip the secondary configurations")
    ap.add_argument("--secondary", default="",
                    help="N = 1: comma-separated subset of the secondary entries to run "
                         "(default: all)")
    ap.add_argument("--single-batch", action="store_true",
                    help="time one batch over and over instead of alternating two")
    ap.add_argument("--n-fft", type=int, choices=(512, 1024), default=1024,
                    help="STFT size (hop n/2); 1024 is the BASELINE configs, 512 oracle_debug's default")
    ap.add_argument("--unet-dtype", choices=("fp32", "bf16"), default="fp32",
                    help="unet workload: U-Net forward precision (fp32 = the reference's)")
    ap.add_argument("--normalize", choices=("peak", "deferred"), default="peak",
                    help="ibm/ipd: peak normalisation in HBM (the reference's output, the "
                         "headline) or deferred to the consumer (the batch driver's form: "
                         "un-normalised output + peak[B], no rescale pass)")
    ap.add_argument("--scenes", choices=("philox", "host"), default="philox",
                    help="input scenes: generated on the device (avz_scene_generate) or the "
                         "host numpy generator (make_batch)")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="N > 1 rehearsal on one GPU: all ranks on cuda:0, gloo collectives")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-kernel HIP events (roofline from the step events)")
    ap.add_argument("--ibm-kappa", type=float, default=0.0,
                    help="diagnostic: the IBM plans' certificate constant (avz_config.ibm_kappa; "
                         "0 = the library default, < 0 = fp32 decisions only)")
    ap.add_argument("--no-settle", action="store_true",
                    help="skip the clock-settling steps before the warmup (cold-GPU timing)")
    a = ap.parse_args()
    shard2 = a.workload == "ibm" and a.gpus > 1
    a.batch = a.batch or (512 if shard2 else DEFAULT_BATCH[a.workload])
    a.interferers = a.interferers or (3 if shard2 else 2)
    return a


# ----------------------------------------------------------------------------- CPU baseline
_CPU_SAMPLE = None


def _cpu_worker(args):
    wid, budget, workload, vectorised, n_fft = args
    from threadpoolctl import threadpool_limits

    from oracle import avz_oracle as O
    mix, tgt, itf = _CPU_SAMPLE
    hop = n_fft // 2
    n = 0
    bins = 0
    t0 = time.perf_counter()
    with threadpool_limits(1):
        while time.perf_counter() - t0 < budget:
            b = (wid + n) % mix.shape[0]
            if workload == "ipd":
                O.masked_mvdr_vec(mix[b], n_fft=n_fft, hop=hop)
            elif vectorised:
                O.oracle_debug_vec(mix[b], tgt[b], itf[b], n_fft=n_fft, hop=hop, sigma=1.0)
            else:
                O.oracle_debug_loop(mix[b], tgt[b], itf[b], n_fft=n_fft, hop=hop, sigma=1.0)
            bins += (n_fft // 2 + 1) * O.n_frames(mix.shape[-1], n_fft, hop)
            n += 1
    return n, bins, time.perf_counter() - t0


def cpu_share():
    """Host cores this process may use: the cgroup CPU quota (cpu.max, cgroup v2) when one
    is set, else the affinity mask. On the MI355X boxes the affinity mask lists the whole
    machine while the job's share is CPU_SHARE cores per GPU."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    return affinity, quota


def cpu_baseline(sample, seconds, workers, workload, n_fft, available, quota=None):
    """The oracle restatement of the same path (oracle/avz_oracle.py, kind 'port') on the
    host cores, time-boxed, one single-threaded worker process per core: the
    loop-faithful oracle_debug (ibm) or the vectorised masked_mvdr (ipd)."""
    import multiprocessing as mp
    global _CPU_SAMPLE
    _CPU_SAMPLE = sample
    ctx = mp.get_context("fork")  # forked before any GPU initialisation
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(w, seconds, workload, False, n_fft) for w in range(workers)])
        wall = time.perf_counter() - t0
        # the vectorised restatement is reported beside the loop-faithful one
        vec = None
        if workload == "ibm":
            rv = pool.map(_cpu_worker, [(w, seconds / 2, workload, True, n_fft) for w in range(workers)])
            vec = sum(r[1] for r in rv) / max(r[2] for r in rv)
    utts = sum(r[0] for r in res)
    bins = sum(r[1] for r in res)
    value = bins / max(r[2] for r in res)
    what = ("vectorised restatement of masked_mvdr.main (IPD mask, sigma 1e-7)"
            if workload == "ipd" else
            "loop-faithful restatement of oracle_debug.main (oracle IBM, sigma 1)")
    share = min(CPU_SHARE, available)
    return {"value": value, "unit": "TF-bins/s", "cores": workers,
            "cores_available": share, "affinity_cores": available, "cgroup_cpu_quota": quota,
            "kind": "port", "value_vectorised": vec, "value_per_core": value / workers,
            "value_affinity_cores_extrapolated": value / workers * available,
            "sample": (f"time-boxed {seconds:.0f} s x {workers} single-threaded workers over "
                       f"{sample[0].shape[0]} distinct utterances of the same workload (4.0 s, "
                       f"{n_fft}/{n_fft // 2}): {utts} utterances; {what} minus WAV I/O; wall "
                       f"{wall:.1f} s; cores_available = the job's CPU share per GPU on the "
                       f"MI355X boxes ({CPU_SHARE}; the affinity mask lists the machine's "
                       f"{available}, and the boxes' rules size worker pools to the share); "
                       "value_affinity_cores_extrapolated = value_per_core x affinity_cores, "
                       "the figure all affinity cores would reach at linear scaling"
                       + ("; value_vectorised: the vectorised restatement (oracle_debug_vec), "
                          "same workers, half the time box" if vec is not None else ""))}


# ----------------------------------------------------------------------------- workloads
TIMING_PERIOD = 4  # timed steps per HIP-event-bracketed analysis launch
UNET_SECONDARY_STEPS = 2  # configs[4] end to end in the default run: ~1.4 s per step
SETTLE_BLOCK = 20  # steps per clock-settling block
SETTLE_MIN_S = 0.1  # sustained load before the convergence test (the clock ramps for tens of ms)
SETTLE_MAX_S = 0.6  # cap on the settling phase


def bytes_per_bin(workload, n_fft):
    """every 4-byte sample stream costs 4 H / F B per TF-bin (3.992 at
    1024/512). ibm: 2 mic + 2 references + output = 19.96 B/bin; ipd: 2 mic + output =
    11.98; external mask: + 4 B/bin of mask = 15.98."""
    per_stream = 4.0 * (n_fft // 2) / (n_fft // 2 + 1)
    return {"ibm": 5 * per_stream, "ipd": 3 * per_stream,
            "unet": 3 * per_stream + 4.0, "chain4": 3 * per_stream + 4.0}[workload]


def gen_batch(spec, dev, start, scenes):
    import torch

    from avz import synth
    S = int(SECONDS * FS)
    if scenes == "philox":
        return synth.make_batch_device(spec["B"], start=start, n_samples=S,
                                       n_interferers=spec["k"], device=dev, rng="philox")
    hm, ht, hi = synth.make_batch(spec["B"], start=start, n_samples=S, n_interferers=spec["k"])
    return tuple(torch.from_numpy(a).to(dev) for a in (hm, ht, hi))


def setup_chain(spec, dev, batches):
    """ibm / ipd: one avz_mvdr_batch call per step (inputs already resident in HBM), the
    steps alternating over the batches."""
    import torch

    import avz
    B, n_fft, S = spec["B"], spec["n_fft"], int(SECONDS * FS)
    hop = n_fft // 2
    norm = "peak" if spec["normalize"] == "peak" else "none"
    if spec["workload"] == "ibm":
        plan = avz.MVDRPlan(n_fft=n_fft, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                            normalize=norm, max_batch=B, max_samples=S,
                            ibm_kappa=spec.get("ibm_kappa", 0.0))
        streams = 4
    else:
        plan = avz.MVDRPlan(n_fft=n_fft, sigma=1e-7, mic_d=0.01, mask="ipd", postfilter="none",
                            normalize=norm, norm_eps=1e-6, max_batch=B, max_samples=S)
        streams = 2
    lens = torch.full((B,), S, dtype=torch.int32, device=dev)
    sets = []
    for d_mix, d_tgt, d_itf in batches:
        refs = dict(ref_tgt=d_tgt, ref_int=d_itf) if spec["workload"] == "ibm" else {}
        sets.append(dict(mix=d_mix, refs=refs, out=plan.alloc_out(B, S, dev),
                         peak=torch.empty((B,), dtype=torch.float32, device=dev)))
    it = [0]

    def step():
        s = sets[it[0] % len(sets)]
        it[0] += 1
        plan.run(s["mix"], lens, max_len=S, out=s["out"], peak=s["peak"], **s["refs"])

    n_out = plan.out_len(S)
    F, T = n_fft // 2 + 1, -(-S // hop) + 1
    nch = -(-T // 32)
    s0 = sets[0]
    ibm = spec["workload"] == "ibm"
    # per-kernel compulsory bytes (synthesis: the output stream) and the recompute design's
    # bytes (+ the mixture re-read, the IBM words and the covariance partials it reads)
    alg_syn = B * n_out * 4
    design_syn = alg_syn + B * 2 * S * 4 + B * nch * F * 4 * (5 + (1 if ibm else 0))
    syn_name = (f"avz_synthesis_utt{'' if n_fft == 1024 else '512'}_kernel"
                f"<{'IBM' if ibm else 'NONE'}, solve fused> (per utterance; chunk-grid "
                "avz_synthesis_kernel for batches routed to it)")
    info = dict(plan=plan, out=s0["out"][:, :min(n_out, S)], peak=s0["peak"], bins=B * F * T,
                alg_analysis=B * streams * S * 4, alg_chain=B * (streams * S * 4 + n_out * 4),
                kernel=f"avz_analysis_kernel<{n_fft},{'IBM' if ibm else 'IPD'}>",
                alg_kernel={"synthesis": alg_syn, "finalize": alg_syn},
                design_kernel={"synthesis": design_syn, "finalize": 2 * alg_syn},
                kernel_names={"synthesis": syn_name, "solve": f"avz_solve_kernel<{n_fft}>",
                              "finalize": f"avz_finalize_kernel<{n_fft}>"},
                mix=s0["mix"], refs=s0["refs"], sets=sets, it=it)
    return step, info


def setup_unet(spec, dev, batches, unet_dtype):
    import torch

    from avz import neural as N
    torch.manual_seed(20250101)
    model = N.FreqPreservingUNet().eval().to(dev)
    B, S = spec["B"], int(SECONDS * FS)
    n_items = B * -(-S // 16000)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[unet_dtype]
    bf = N.NeuralMaskBeamformer(model, max_items=n_items, model_dtype=dt)
    y = {}
    it = [0]

    def step():
        d_mix = batches[it[0] % len(batches)][0]
        it[0] += 1
        y["out"], _ = bf.run(d_mix)

    n_fft = spec["n_fft"]
    F = n_fft // 2 + 1
    Tc = -(-bf.chunk // (n_fft // 2)) + 1
    n_out = bf.plan.out_len(bf.chunk)
    info = dict(plan=bf.plan, bf=bf, bins=n_items * F * Tc, n_items=n_items,
                alg_analysis=n_items * 2 * bf.chunk * 4,
                alg_chain=n_items * (2 * bf.chunk * 4 + n_out * 4),
                kernel=f"avz_analysis_kernel<{n_fft},EXTERNAL>", mix=batches[0][0], y=y, it=it)
    return step, info


def conv_flops(model, x):
    """FLOPs of one forward of `model` on x (2 per multiply-add of every Conv2d /
    ConvTranspose2d, counted by hooks on a forward of x)."""
    import torch
    tot = [0]

    def hook(mod, inp, out):
        k = mod.weight.shape  # Conv2d [cout, cin/g, kh, kw]; ConvTranspose2d [cin, cout/g, kh, kw]
        if isinstance(mod, torch.nn.ConvTranspose2d):
            tot[0] += 2 * inp[0].numel() * k[1] * k[2] * k[3]
        else:
            tot[0] += 2 * out.numel() * k[1] * k[2] * k[3]
    hs = [m.register_forward_hook(hook) for m in model.modules()
          if isinstance(m, (torch.nn.Conv2d, torch.nn.ConvTranspose2d))]
    with torch.no_grad():
        model(x)
    for h in hs:
        h.remove()
    return tot[0]


def unet_figures(info, K, chain_ms):
    """configs[4]'s parts, timed alone on the same items: the U-Net forward (device features
    included) with its achieved TFLOP/s against the fp32 peak, and the MVDR chain."""
    import torch
    bf = info["bf"]
    items = bf.split(info["mix"])[0]
    from avz import neural as N
    x = N.mask_features(bf.plan, items[:1], "unet")
    if bf.channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    flops_chunk = conv_flops(bf.model, x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(1, K // 2)
    e0.record()
    for _ in range(n):
        bf.masks(items)
    e1.record()
    torch.cuda.synchronize()
    unet_ms = e0.elapsed_time(e1) / n
    tflops = flops_chunk * info["n_items"] / (unet_ms * 1e-3) / 1e12
    return {"unet_ms": unet_ms, "mvdr_chain_ms": chain_ms,
            "mvdr_chain_tf_bins_per_s": info["bins"] / (chain_ms * 1e-3),
            "unet_gflop_per_chunk": flops_chunk / 1e9, "unet_tflops": tflops,
            "unet_frac_fp32_peak": tflops / FP32_PEAK_TFLOPS,
            "unet_note": ("U-Net forward incl. device features, torch events around masks() on "
                          "the batch's chunk items; FLOPs = 2 x MACs of every convolution")}


def setup_chain4(spec, dev, batches):
    """configs[4]'s MVDR chain alone: the batch's 2-s chunk items (avz_chunk_split) through
    the external-mask chain with a fixed synthetic target mask (what the U-Net would hand
    over), one avz_mvdr_batch call per step."""
    import torch

    from avz import neural as N
    bf = N.NeuralMaskBeamformer(torch.nn.Identity(), max_items=spec["B"] * 4)
    sets = []
    for d_mix, _, _ in batches:
        items = bf.split(d_mix)[0]
        F, T = bf.plan.cfg.n_fft // 2 + 1, bf.plan.frames(bf.chunk)
        g = torch.Generator(device=dev).manual_seed(7)
        mask = torch.rand((items.shape[0], F, T), generator=g, device=dev)
        n = items.shape[0]
        sets.append(dict(items=items, mask=mask, out=bf.plan.alloc_out(n, bf.chunk, dev),
                         peak=torch.empty((n,), dtype=torch.float32, device=dev),
                         lens=torch.full((n,), bf.chunk, dtype=torch.int32, device=dev)))
    it = [0]

    def step():
        s = sets[it[0] % len(sets)]
        it[0] += 1
        bf.plan.run(s["items"], s["lens"], max_len=bf.chunk, ext_mask=s["mask"], out=s["out"],
                    peak=s["peak"])

    n = sets[0]["items"].shape[0]
    F, T = bf.plan.cfg.n_fft // 2 + 1, bf.plan.frames(bf.chunk)
    n_out = bf.plan.out_len(bf.chunk)
    info = dict(plan=bf.plan, bins=n * F * T, n_items=n, alg_analysis=n * 2 * bf.chunk * 4,
                alg_chain=n * (2 * bf.chunk * 4 + n_out * 4 + F * T * 4),
                kernel=f"avz_analysis_kernel<{bf.plan.cfg.n_fft},EXTERNAL>", it=it)
    return step, info


# avz_beamform_spectral (batch_mvdr on a held STFT, tf_lite_version/inference.py:85-179, with
# the driver's S * max(M, 0.05) fused): Y 2 x 8 B + mask 4 B read, S 8 B written per TF-bin
SPECTRAL_BYTES_PER_BIN = 28


def setup_spectral(n_items, dev, n_sets):
    """avz_beamform_spectral over n_items 2-s chunk spectra ([2, 513, 64] complex64 Y, a
    [513, 64] target mask) per step, the steps alternating over n_sets input sets."""
    import torch

    from avz import spectral
    F, T = 513, 64
    sb = spectral.SpectralBeamformer("mvdr", max_items=n_items, floor=0.05)
    g = torch.Generator(device=dev).manual_seed(11)
    sets = []
    for _ in range(n_sets):
        Y = torch.view_as_complex(torch.randn((n_items, 2, F, T, 2), generator=g, device=dev))
        M = torch.rand((n_items, F, T), generator=g, device=dev)
        sets.append((Y, M, torch.empty((n_items, F, T), dtype=torch.complex64, device=dev)))
    it = [0]

    def step():
        Y, M, S = sets[it[0] % len(sets)]
        it[0] += 1
        sb.beamform(Y, M, S=S)

    return step, dict(plan=sb.plan, bins=n_items * F * T, it=it,
                      kernel="avz_spectral_kernel<1024,MVDR,EXT_FLOOR> (+ batch-fallback fixup)")


SWEEP_B = (1, 64, 200, 255, 256, 257, 300, 384)  # configs[1]'s chain at other batch sizes


def batch_sweep(dev, args, n_sets, K, W):
    """configs[1]'s chain (4.0 s, 2 interferers, oracle IBM, 1024/512, peak normalisation)
    at the batch sizes of SWEEP_B, measured as the headline: value, ms per step, the kernels'
    ms, and the rate relative to B = 256 (all utterances are 4.0 s, so TF-bins/s is
    proportional to utterances/s). The reference's batch driver takes any --n
    (Final_pipeline/batch_run.py:12,53, default 10)."""
    import torch
    res = {}
    for B in SWEEP_B:
        try:
            sp = dict(workload="ibm", B=B, k=2, n_fft=1024, normalize="peak")
            bs = [gen_batch(sp, dev, i * B, args.scenes) for i in range(n_sets)]
            st, inf = setup_chain(sp, dev, bs)
            el, ktx, _ = run_timed(st, inf["plan"], K, W, 1, dev, not args.no_settle,
                                   not args.no_kernel_timing)
            e = {"value": inf["bins"] * K / el, "ms_per_step": 1e3 * el / K,
                 "tf_bins_per_step": inf["bins"]}
            if ktx:
                e["kernels_ms"] = {k: ktx[k] for k in inf["plan"].KERNELS}
            res[str(B)] = e
            del bs, st, inf
            torch.cuda.empty_cache()
        except Exception as exc:  # a side figure must never sink the bench line
            res[str(B)] = {"error": repr(exc)[:300]}
    ref = res.get("256", {}).get("value")
    if ref:
        for e in res.values():
            if "value" in e:
                e["rate_vs_b256"] = e["value"] / ref
        ge = [e["rate_vs_b256"] for b, e in res.items() if int(b) >= 256 and "value" in e]
        res["min_rate_vs_b256_for_b_ge_256"] = min(ge) if ge else None
    res["config"] = ("configs[1] chain at batch B in " + str(list(SWEEP_B)) + ": 4.0 s, 2 "
                     "interferers, oracle IBM, 1024/512, peak normalisation; rate_vs_b256 = "
                     "value / value at B = 256")
    return res


def configs0_latency(dev, n_calls=50):
    """configs[0]: ONE mixture through oracle_debug (rt_av_zoom/core/oracle_debug.py:27-97),
    the bundled 8.23-s test triple (tests/golden/inputs_test.npz, int16 / 32768 as the
    reference reads it), at 512/256 (as shipped) and 1024/512, sigma 1: the engine's time per
    call (back to back, and call + synchronize as a real-time caller sees it) beside the
    loop-faithful CPU oracle on the same triple (one core), and the output's SIR against the
    reference-run golden (full_test_n{N}_s1.npz)."""
    import torch
    from threadpoolctl import threadpool_limits

    import avz
    from oracle import avz_oracle as O
    gdir = os.path.join(ROOT, "tests", "golden")
    with np.load(os.path.join(gdir, "inputs_test.npz"), allow_pickle=False) as z:
        f = lambda a: (a.astype(np.float64) / 32768.0).astype(np.float32)  # noqa: E731
        mix, tgt, itf = f(z["mix"]).T.copy(), f(z["tgt"]), f(z["int"])
    S = len(tgt)
    res = {"config": ("configs[0]: one mixture (bundled test triple, 8.23 s, 1 interferer), "
                      "oracle IBM, sigma 1, B = 1"), "samples": S}
    for n in (512, 1024):
        plan = avz.MVDRPlan(n_fft=n, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                            normalize="peak", max_batch=1, max_samples=S)
        d_mix = torch.from_numpy(mix).to(dev)[None]
        d_t, d_i = torch.from_numpy(tgt).to(dev)[None], torch.from_numpy(itf).to(dev)[None]
        lens = torch.full((1,), S, dtype=torch.int32, device=dev)
        out = plan.alloc_out(1, S, dev)
        peak = torch.empty((1,), dtype=torch.float32, device=dev)

        def call():
            plan.run(d_mix, lens, max_len=S, out=out, peak=peak, ref_tgt=d_t, ref_int=d_i)
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_calls):
            call()
        torch.cuda.synchronize()
        pipelined = 1e3 * (time.perf_counter() - t0) / n_calls
        lat = []
        for _ in range(n_calls):
            t0 = time.perf_counter()
            call()
            torch.cuda.synchronize()
            lat.append(1e3 * (time.perf_counter() - t0))
        plan.set_timing(True)
        for _ in range(10):
            call()
        kt = plan.timing()
        plan.set_timing(False)
        # the round-3 synthesis form for comparison: chunk grid + solve + finalize launches
        # (the plan's diagnostics, synth_variant 0; the analysis kernel as above)
        alt = None
        if True:
            plan.set_diagnostics(synth_variant=0)
            try:
                for _ in range(10):
                    call()
                torch.cuda.synchronize()
                lat0 = []
                for _ in range(n_calls):
                    t0 = time.perf_counter()
                    call()
                    torch.cuda.synchronize()
                    lat0.append(1e3 * (time.perf_counter() - t0))
                alt = float(np.median(lat0))
            finally:
                plan.set_diagnostics(synth_variant=2)
        call()
        torch.cuda.synchronize()
        n_out = plan.out_len(S)
        got = out[0, :n_out].cpu().numpy().astype(np.float64)
        with np.load(os.path.join(gdir, f"full_test_n{n}_s1.npz"), allow_pickle=False) as g:
            sir_ref = float(g["sir_out"])
        L = min(len(got), S)
        sir = O.projection_sdr_sir(got[:L], tgt[:L], itf[:L])[1]
        with threadpool_limits(1):
            cpu = []
            for _ in range(3):
                t0 = time.perf_counter()
                O.oracle_debug_loop(mix, tgt, itf, n_fft=n, hop=n // 2, sigma=1.0)
                cpu.append(1e3 * (time.perf_counter() - t0))
        F, T = n // 2 + 1, O.n_frames(S, n, n // 2)
        res[f"n{n}"] = {
            "ms_per_call_back_to_back": pipelined,
            "ms_per_call_synchronous_median": float(np.median(lat)),
            "ms_per_call_synchronous_p90": float(np.percentile(lat, 90)),
            "kernels_ms": {k: kt[k] for k in plan.KERNELS},
            "tf_bins": F * T, "tf_bins_per_s_back_to_back": F * T / (pipelined * 1e-3),
            "sir_out_db": float(sir), "sir_out_reference_db": sir_ref,
            "sir_abs_delta_db": abs(float(sir) - sir_ref),
            "ms_per_call_synchronous_chunk_grid_synthesis": alt,
            "cpu_oracle_loop_ms_median_1core": float(np.median(cpu)),
            "speedup_vs_cpu_1core_synchronous": float(np.median(cpu) / np.median(lat))}
        del plan
    return res


def run_timed(step, plan, K, W, world, dev, settle_on, kernel_timing):
    """Clock settling, W warmup steps, K timed steps (barrier + synchronize on both sides),
    then an untimed pass with HIP events around all four kernels."""
    import torch
    import torch.distributed as dist
    # Clock settling: a GPU that sat idle (host scene setup, the CPU baseline) runs its
    # compute-bound kernels 10-15 % slower for the first tens of milliseconds of load
    # (profiles/r02u/warmup_sensitivity.txt). Untimed blocks of SETTLE_BLOCK steps run for at
    # least SETTLE_MIN_S and until two consecutive blocks agree within 1 % (at most
    # SETTLE_MAX_S), so the K timed steps measure the steady state a continuous job runs at;
    # the first block's per-step time is reported as settle.cold_ms_per_step.
    settle = {"steps": 0, "ms": 0.0, "cold_ms_per_step": None}
    if settle_on:
        s0 = time.perf_counter()
        step()  # first launch (code objects, attributes) outside the cold measurement
        settle["steps"] = 1
        prev = None
        while True:
            torch.cuda.synchronize()
            b0 = time.perf_counter()
            for _ in range(SETTLE_BLOCK):
                step()
            torch.cuda.synchronize()
            per = (time.perf_counter() - b0) / SETTLE_BLOCK
            settle["steps"] += SETTLE_BLOCK
            if settle["cold_ms_per_step"] is None:
                settle["cold_ms_per_step"] = 1e3 * per
            done = (prev is not None and abs(per - prev) <= 0.01 * prev
                    and time.perf_counter() - s0 >= SETTLE_MIN_S)
            prev = per
            if done or time.perf_counter() - s0 > SETTLE_MAX_S:
                break
        settle["ms"] = 1e3 * (time.perf_counter() - s0)
    for _ in range(W):
        step()
    torch.cuda.synchronize()

    if kernel_timing:
        plan.set_timing(True, analysis_only=True, period=TIMING_PERIOD)
    # No torch events inside the timed loop: a default torch.cuda.Event record is a
    # system-scope release (an L2 writeback, ~15 us between steps on MI355X). The plan's
    # own events (hipEventDisableSystemFence, carried by the kernel's dispatch) bracket the
    # dominant (analysis) kernel on every TIMING_PERIOD-th timed step only: even those cost
    # ~7 us per bracketed step (profiles/r02t/timing_overhead.txt), so the steps in between
    # run exactly as an untimed caller's would.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    kt = None
    if kernel_timing:
        dom = plan.timing()  # the bracketed steps among the K timed ones
        plan.set_timing(True)  # every kernel of the chain: a separate, untimed pass
        for _ in range(max(3, K // 4)):
            step()
        kt = plan.timing()
        plan.set_timing(False)
        kt["analysis_timed"] = dom["analysis"]
        kt["analysis_timed_calls"] = dom["calls"]
    return t1 - t0, kt, settle


def sq_busy(kernel_prefix, n_cu, batch):
    """VALU / LDS busy fractions of a kernel from profiles/pmc_sq.json (tools/pmc_sq.sh on this
    configuration, B = batch), or {} when there is none."""
    path = os.path.join(ROOT, "profiles", "pmc_sq.json")
    if not os.path.exists(path):
        return {}
    doc = json.load(open(path))
    if doc.get("batch") != batch:
        return {}
    for k, c in doc.get("kernels", {}).items():
        if k.startswith(kernel_prefix) and c.get("GRBM_GUI_ACTIVE"):
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0
            r = {"sq_source": doc.get("source"), "sq_kernel": k}
            if "SQ_ACTIVE_INST_VALU" in c:
                r["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4.0 / (4.0 * n_cu) / cyc
            if "SQ_LDS_IDX_ACTIVE" in c:
                r["lds_busy"] = c["SQ_LDS_IDX_ACTIVE"] / n_cu / cyc
            return r
    return {}


def secondary_entry(spec, info, K, elapsed, kt, world):
    """A secondary configuration's figures, measured as the headline's; its dominant kernel
    is the longest of the untimed all-kernel pass, as the headline's."""
    value = world * info["bins"] * K / elapsed
    bpb = bytes_per_bin(spec["workload"], spec["n_fft"])
    e = {"config": spec["text"], "value": value, "unit": "TF-bins/s",
         "ms_per_step": 1e3 * elapsed / K,
         "frac": value / world * bpb / 1e9 / HBM_PEAK_GBS, "bytes_per_bin": bpb,
         "tf_bins_per_step": info["bins"]}
    if kt:
        plan = info["plan"]
        e["kernels_ms"] = {k: kt[k] for k in plan.KERNELS}
        name = max(plan.KERNELS, key=lambda k: kt[k] if kt[k] == kt[k] else -1.0)
        if name == "analysis":
            dom_ms = kt["analysis_timed"]
            e["dominant_kernel"] = {"kernel": info["kernel"], "role": name, "kernel_ms": dom_ms,
                                    "frac": info["alg_analysis"] / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        else:
            ms = kt[name]
            alg = info.get("alg_kernel", {}).get(name, 0)
            e["dominant_kernel"] = {"kernel": info.get("kernel_names", {}).get(name, name),
                                    "role": name, "kernel_ms": ms,
                                    "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    return e


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    S = int(SECONDS * FS)
    B = args.batch
    N_FFT, HOP = args.n_fft, args.n_fft // 2

    from avz import synth
    gen_host = synth.make_batch_philox if args.scenes == "philox" else synth.make_batch

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.workload != "unet":
        available, quota = cpu_share()
        share = min(CPU_SHARE, available)
        if quota is not None:
            share = max(1, min(share, int(quota)))
        workers = args.cpu_workers or share
        k = min(B, 32)
        # the host restatement of the same scenes (forked before any GPU initialisation)
        sample = gen_host(k, start=rank * B, n_samples=S, n_interferers=args.interferers)
        cpu = cpu_baseline(sample, args.cpu_seconds, workers, args.workload, N_FFT, available,
                           quota)

    import torch
    import torch.distributed as dist

    from avz import metrics
    from avz.batch_run import allreduce_job, finite_sums
    from oracle import avz_oracle as O

    # --rehearse-shared-gpu: every rank on cuda:0 with gloo, to exercise the N > 1 code
    # path (sharding, metric all-reduce, max-over-ranks timing) on a one-GPU box
    gpu = 0 if args.rehearse_shared_gpu else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.rehearse_shared_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    spec = dict(workload=args.workload, B=B, k=args.interferers, n_fft=N_FFT,
                normalize=args.normalize, ibm_kappa=args.ibm_kappa)
    # this rank's shard(s) of utterances, generated in HBM: batch 0 = utterances rank * B ..
    # rank * B + B - 1 (the one the SIR metrics score), batch 1 = the next world * B
    g0 = time.perf_counter()
    n_sets = 1 if args.single_batch else 2
    batches = [gen_batch(spec, dev, i * world * B + rank * B, args.scenes) for i in range(n_sets)]
    torch.cuda.synchronize()
    gen_ms = 1e3 * (time.perf_counter() - g0)
    d_mix, d_tgt, d_itf = batches[0]

    if args.workload == "unet":
        step, info = setup_unet(spec, dev, batches, args.unet_dtype)
    else:
        step, info = setup_chain(spec, dev, batches)
    plan = info["plan"]
    K = args.steps
    # a U-Net step alone takes ~1.4 s: no settling blocks for it
    elapsed_s, kt, settle = run_timed(step, plan, K, args.warmup, world, dev,
                                      not args.no_settle and args.workload != "unet",
                                      not args.no_kernel_timing)
    elapsed = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    step_ms = 1e3 * elapsed_s / K
    chain_ms = sum(kt[k] for k in plan.KERNELS) if kt else step_ms

    extra = {}
    if args.workload == "unet":  # the U-Net forward alone (features included), same items
        extra.update(unet_figures(info, K, chain_ms))

    if args.workload != "unet" and rank == 0:
        try:
            # PCIe-inclusive rate (not `value`): the same step with its inputs copied from
            # pinned host memory first and the output copied back (host-buffer callers, e.g.
            # the oracle_debug.main mirror). Reported beside the HBM-resident number.
            pin = lambda x: x.cpu().pin_memory()  # noqa: E731
            ho = torch.empty(tuple(info["out"].shape), dtype=torch.float32).pin_memory()
            d_in = [(pin(info["mix"]), info["mix"])]
            if info["refs"]:
                d_in += [(pin(info["refs"]["ref_tgt"]), info["refs"]["ref_tgt"]),
                         (pin(info["refs"]["ref_int"]), info["refs"]["ref_int"])]
            n_pcie = max(2, K // 4)
            torch.cuda.synchronize()
            p0 = time.perf_counter()
            for _ in range(n_pcie):
                info["it"][0] = 0  # batch 0: the buffers being refilled
                for h, d in d_in:
                    d.copy_(h, non_blocking=True)
                step()
                ho.copy_(info["out"], non_blocking=True)
            torch.cuda.synchronize()
            pcie_ms = 1e3 * (time.perf_counter() - p0) / n_pcie
            h2d = sum(h.numel() * 4 for h, _ in d_in)
            extra["pcie_inclusive"] = {"ms_per_step": pcie_ms,
                                       "tf_bins_per_s": info["bins"] / (pcie_ms * 1e-3),
                                       "h2d_bytes": h2d, "d2h_bytes": ho.numel() * 4,
                                       "note": "rank 0; not the headline value"}
        except Exception as exc:  # a side figure must never sink the bench line
            extra["pcie_inclusive"] = {"error": repr(exc)[:200]}

    # ---- final metrics: projection SIR per utterance (run_metrics.py:6-36), RCCL all-reduce
    # of batch 0's outputs: one more step on batch 0 leaves them in its output buffer
    info["it"][0] = 0
    step()
    torch.cuda.synchronize()
    L = S
    if args.workload == "unet":
        est_out = info["y"]["out"][:, :L]
    else:
        est_out = info["out"][:, :L]
        L = est_out.shape[1]
    d_tgt, d_itf = d_tgt[:, :L], d_itf[:, :L]
    est = torch.cat([est_out, d_mix[:, 0, :L]])
    est_peak = None
    if args.workload != "unet" and args.normalize == "deferred":  # score out / peak
        eps = 1e-6 if args.workload == "ipd" else 0.0
        est_peak = torch.cat([info["peak"] + eps, torch.ones_like(info["peak"])])
    m = metrics.projection_metrics(est, torch.cat([d_tgt] * 2), torch.cat([d_itf] * 2),
                                   est_peak=est_peak)
    sir_out, sir_in = m[:B, 3], m[B:, 3]
    # [sum SIR_in, sum SIR_out, sum OSINR_out, n_ok, n] over the utterances
    # whose metrics are finite (batch_run.finite_sums)
    sums = finite_sums([sir_in, sir_out, m[:B, 0]], B)
    if world > 1:  # SUM of the metric sums, MAX over ranks of the timings
        kn = plan.KERNELS + ("analysis_timed",)
        mx = torch.tensor([elapsed_s, step_ms, chain_ms] + ([kt[k] for k in kn] if kt else []),
                          dtype=torch.float64, device=dev)
        allreduce_job(sums, mx)
        elapsed = mx[:1]
        step_ms, chain_ms = float(mx[1]), float(mx[2])
        if kt:
            kt.update({k: float(mx[3 + j]) for j, k in enumerate(kn)})
    # SIR delta vs the reference restatement on identical inputs (rank 0, few utterances)
    d_sir = None
    if rank == 0 and args.workload != "unet":
        k = min(B, 4)
        got = sir_out[:k].cpu().numpy()
        mix, tgt, itf = (x[:k].cpu().numpy() for x in (d_mix, d_tgt, d_itf))
        refs = []
        for b in range(k):
            if args.workload == "ipd":
                r = O.masked_mvdr_vec(mix[b], n_fft=N_FFT, hop=HOP)
            else:
                r = O.oracle_debug_vec(mix[b], tgt[b], itf[b], n_fft=N_FFT, hop=HOP, sigma=1.0)
            refs.append(O.projection_sdr_sir(r[:L], tgt[b, :L], itf[b, :L])[1])
        d_sir = float(np.max(np.abs(got - np.array(refs))))

    t_max = float(elapsed.item())
    value = world * info["bins"] * K / t_max
    # Roofline, SURVEY 8(d): achieved = TF-bins/s x bytes_per_bin, per GPU (peak is per GPU).
    bpb = bytes_per_bin(args.workload, N_FFT)
    alg_analysis, alg_chain = info["alg_analysis"], info["alg_chain"]
    traffic = {}
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf) and args.workload == "ibm":
        pm = json.load(open(tf))
        if pm.get("batch") == B and pm.get("n_fft") == N_FFT and pm.get("samples") == S:
            key = "hbm_bytes_per_launch" if args.normalize == "peak" else "deferred_hbm_bytes_per_launch"
            traffic = pm.get(key, {})
            if not isinstance(traffic, dict):
                traffic = {}
    achieved = value / world * bpb / 1e9
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic.get("chain"),
            "bytes_per_bin": bpb,
            "formula": "SURVEY 8(d): value / n_gpus x bytes_per_bin / 8e12",
            "kernel": "avz_mvdr_batch chain (analysis + solve + synthesis + finalize)",
            "kernel_ms": chain_ms, "alg_bytes_per_launch": info["bins"] * bpb}
    if kt:
        dom_ms = kt["analysis_timed"]  # HIP events on the launch stream, over the timed steps
        roof["kernels_ms"] = {k: kt[k] for k in plan.KERNELS}  # separate untimed pass
        roof["kernels_ms_note"] = ("kernels_ms: the four kernels in an untimed pass after the "
                                   "timed steps; analysis_kernel.kernel_ms: the analysis kernel "
                                   f"on every {TIMING_PERIOD}th timed step "
                                   f"({kt['analysis_timed_calls']} of {K} launches), HIP events "
                                   "carried by its dispatch on the launch stream")
        ana = {"kernel": info["kernel"], "kernel_ms": dom_ms,
               "alg_bytes_per_launch": alg_analysis,
               "achieved": alg_analysis / (dom_ms * 1e-3) / 1e9,
               "frac": alg_analysis / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
               "traffic": traffic.get("analysis")}
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        ana.update(sq_busy("avz_analysis_kernel", n_cu, B))
        roof["analysis_kernel"] = ana
        # the kernel that bounds the step: the longest of the untimed pass
        name = max(plan.KERNELS, key=lambda k: kt[k] if kt[k] == kt[k] else -1.0)
        if name == "analysis":
            roof["dominant_kernel"] = dict(ana, role="analysis")
        else:
            ms = kt[name]
            alg = info["alg_kernel"].get(name, 0)
            design = info["design_kernel"].get(name, alg)
            roof["dominant_kernel"] = {
                "kernel": info["kernel_names"].get(name, name), "role": name, "kernel_ms": ms,
                "alg_bytes_per_launch": alg,
                "achieved": alg / (ms * 1e-3) / 1e9,
                "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "design_bytes_per_launch": design,
                "frac_design": design / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "traffic": traffic.get(name),
                **sq_busy(info["kernel_names"].get(name, name).split("<")[0], n_cu, B),
                "note": ("alg: its compulsory bytes (the output stream); design: + the mixture "
                         "re-read of the recompute design (the forward FFT is recomputed "
                         "instead of storing Y), the IBM words and the covariance partials; "
                         "kernel_ms from the untimed all-kernel pass")}
        roof["chain_events"] = {"ms": chain_ms, "alg_bytes_per_launch": alg_chain,
                                "achieved": alg_chain / (chain_ms * 1e-3) / 1e9,
                                "frac": alg_chain / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}

    # ---- the other single-GPU configurations, same method, same line (N = 1 default run)
    secondary = None
    default_run = (args.workload == "ibm" and N_FFT == 1024 and B == 256 and args.interferers == 2
                   and args.normalize == "peak")
    if world == 1 and default_run and not args.no_secondary:
        del batches, d_mix, d_tgt, d_itf, est, m, info, step
        torch.cuda.empty_cache()
        secondary = {}
        specs = [
            ("configs[2]_shard", dict(workload="ibm", B=512, k=3, n_fft=1024, normalize="peak",
                                       text="configs[2] per-GPU shard: B=4096 over 8 GPUs = 512 "
                                            "utterances, 3 interferers, oracle IBM, 1024/512")),
            ("configs[3]", dict(workload="ipd", B=1024, k=2, n_fft=1024, normalize="peak",
                                text="configs[3]: B=1024, heuristic IPD mask, sigma 1e-7, no "
                                     "post-filter, 1024/512")),
            ("n_fft_512", dict(workload="ibm", B=256, k=2, n_fft=512, normalize="peak",
                               text="configs[1] at oracle_debug's 512/256 STFT (Fft512x2)")),
            ("deferred_norm", dict(workload="ibm", B=256, k=2, n_fft=1024, normalize="deferred",
                                   text="configs[1], the batch driver's deferred normalisation "
                                        "(un-normalised output + peak[B])")),
            ("configs[4]_chain", dict(workload="chain4", B=1024, k=2, n_fft=1024, normalize="none",
                                      text=WORKLOAD_TEXT["chain4"].format(B=1024, n=1024, h=512))),
            ("configs[4]_unet", dict(workload="unet", B=1024, k=2, n_fft=1024, normalize="none",
                                     text=WORKLOAD_TEXT["unet"].format(B=1024, unet_dtype="fp32",
                                                                       n=1024, h=512))),
        ]
        only = set(x for x in args.secondary.split(",") if x)
        want = lambda name: not only or name in only  # noqa: E731
        if want("configs[0]_latency"):
            try:
                secondary["configs[0]_latency"] = configs0_latency(dev)
            except Exception as exc:  # a side figure must never sink the bench line
                secondary["configs[0]_latency"] = {"error": repr(exc)[:300]}
            torch.cuda.empty_cache()
        if want("batch_sweep"):
            secondary["batch_sweep"] = batch_sweep(dev, args, n_sets, K, args.warmup)
        specs = [x for x in specs if want(x[0])]
        try:  # the spectral-domain operator on a 4096-item chunk batch (configs[4]'s items)
            if not want("spectral_4096"):
                raise StopIteration
            st, inf = setup_spectral(4096, dev, n_sets)
            el, _, _ = run_timed(st, inf["plan"], K, args.warmup, 1, dev, not args.no_settle,
                                 False)
            v = inf["bins"] * K / el
            ach = inf["bins"] * SPECTRAL_BYTES_PER_BIN / (el / K) / 1e9
            secondary["spectral_4096"] = {
                "config": "avz_beamform_spectral: 4096 items of [2, 513, 64] complex64 STFT + "
                          "[513, 64] target mask, batch_mvdr semantics (sigma 1e-5, d 0.04, "
                          "item-level singular fallback), S * max(M, 0.05) fused",
                "value": v, "unit": "TF-bins/s", "ms_per_step": 1e3 * el / K,
                "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                             "bytes_per_bin": SPECTRAL_BYTES_PER_BIN,
                             "alg_bytes_per_launch": inf["bins"] * SPECTRAL_BYTES_PER_BIN,
                             "kernel": inf["kernel"],
                             "note": "step wall time / K (both launches of the call)"}}
            del st, inf
            torch.cuda.empty_cache()
        except StopIteration:
            pass
        except Exception as exc:  # a side figure must never sink the bench line
            secondary["spectral_4096"] = {"error": repr(exc)[:300]}
        for name, sp in specs:
            try:
                bs = [gen_batch(sp, dev, i * sp["B"], args.scenes) for i in range(n_sets)]
                if sp["workload"] == "unet":
                    # one U-Net step takes ~1.3-1.4 s: a few steps, no settling blocks
                    Ku = UNET_SECONDARY_STEPS
                    st, inf = setup_unet(sp, dev, bs, "fp32")
                    el, ktx, _ = run_timed(st, inf["plan"], Ku, 1, 1, dev, False,
                                           not args.no_kernel_timing)
                    cm = sum(ktx[k] for k in inf["plan"].KERNELS) if ktx else 1e3 * el / Ku
                    secondary[name] = secondary_entry(sp, inf, Ku, el, ktx, 1)
                    secondary[name].update(unet_figures(inf, Ku, cm))
                    secondary[name]["steps"] = Ku
                elif sp["workload"] == "chain4":
                    st, inf = setup_chain4(sp, dev, bs)
                else:
                    st, inf = setup_chain(sp, dev, bs)
                if sp["workload"] != "unet":
                    el, ktx, _ = run_timed(st, inf["plan"], K, args.warmup, 1, dev,
                                           not args.no_settle, not args.no_kernel_timing)
                    secondary[name] = secondary_entry(sp, inf, K, el, ktx, 1)
                del bs, st, inf
                torch.cuda.empty_cache()
            except Exception as exc:  # a side figure must never sink the bench line
                secondary[name] = {"error": repr(exc)[:300]}

    if rank == 0:
        wtext = WORKLOAD_TEXT[args.workload].format(
            B=B, k=args.interferers, unet_dtype=args.unet_dtype, n=N_FFT, h=HOP)
        if args.workload == "ibm" and args.interferers == 3 and B == 512:
            wtext = ("configs[2] per-GPU shard (B=4096 over 8 GPUs = 512 utterances/GPU): "
                     + wtext.split(": ", 1)[1])
        cfg = {"workload": wtext,
               "batch_per_gpu": B, "global_batch": B * world, "samples": S,
               "n_fft": N_FFT, "hop": HOP, "parallelism":
               f"utterance-sharded x{world}, RCCL metric all-reduce only",
               "input_batches": n_sets}
        if args.workload == "ibm":
            cfg.update(tf_bins_per_utt=info_bins_per(B, N_FFT, S), sigma=1.0, mask="ibm",
                       postfilter="ibm", normalize=args.normalize)
        elif args.workload == "ipd":
            cfg.update(tf_bins_per_utt=info_bins_per(B, N_FFT, S), sigma=1e-7, mask="ipd",
                       postfilter="none", normalize=args.normalize)
        else:
            cfg.update(chunk_items=info["n_items"], tf_bins_per_chunk=info["bins"] // info["n_items"],
                       sigma=1e-5, mask="external (U-Net)", postfilter="max(M, 0.05)",
                       normalize="none", unet_dtype=args.unet_dtype)
        line = {
            "metric": METRIC, "value": value, "unit": "TF-bins/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": 1e3 * t_max / K,
            "settle": settle,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic speech-like 2-mic far-field mixtures (SURVEY 8(d) model), "
                     + ("generated in HBM by avz_scene_generate (Philox draws keyed by utterance "
                        f"index; {n_sets} batches of B per rank alternating over the timed steps; "
                        f"{gen_ms:.1f} ms for this rank's)"
                        if args.scenes == "philox" else
                        f"host numpy generator, seeds 1000+idx ({gen_ms:.0f} ms incl. H2D)")),
            "config": cfg,
            "roofline": roof,
            "cpu_baseline": cpu,
            "sir": {"sir_in_mean_db": float(sums[0] / max(float(sums[3]), 1.0)),
                    "sir_out_mean_db": float(sums[1] / max(float(sums[3]), 1.0)),
                    "osinr_out_mean_db": float(sums[2] / max(float(sums[3]), 1.0)),
                    "sir_abs_delta_vs_reference_db": d_sir, "n_ok": int(sums[3]),
                    "n_utts": int(sums[4])},
        }
        line.update(extra)
        if secondary is not None:
            line["secondary"] = secondary
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def info_bins_per(B, n_fft, S):
    hop = n_fft // 2
    return (n_fft // 2 + 1) * (-(-S // hop) + 1)


if __name__ == "__main__":
    main()
