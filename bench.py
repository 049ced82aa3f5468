"""Headline benchmark: beamformed TF-bins/s of the MVDR hot path on MI355X.

Workload (BASELINE.json configs[1]): per GPU a batch of B = 256 synthetic 2-mic
utterances of 4.0 s (64000 samples @ 16 kHz), 2 interferers, oracle IBM mask,
1024-pt STFT / hop 512 -> F x T = 513 x 126 = 64,638 TF-bins per utterance.
One step = one avz_mvdr_batch call over the whole batch: the analysis (STFT -> IBM ->
masked covariance partials), solve (fp64 MVDR), synthesis (STFT -> apply + IBM
post-filter -> iSTFT/OLA) and finalize (chunk seams, peak normalisation) kernels,
inputs resident in HBM. Per-kernel times come from HIP events the plan records
around each launch on the launch stream (avz_plan_set_timing). Multi-GPU: one process per GPU, utterances
sharded (weak scaling, no data-path collective); the only collective is the final
RCCL all-reduce of the SIR metric sums (and the max-over-ranks step time).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
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
N_FFT, HOP, FS, SECONDS = 1024, 512, 16000, 4.0
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="utterances per GPU")
    ap.add_argument("--interferers", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="time box of the CPU baseline workers")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: min(16, available cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-kernel HIP events (roofline from the step events)")
    return ap.parse_args()


# ----------------------------------------------------------------------------- CPU baseline
_CPU_SAMPLE = None


def _cpu_worker(args):
    wid, budget = args
    from threadpoolctl import threadpool_limits

    from oracle import avz_oracle as O
    mix, tgt, itf = _CPU_SAMPLE
    n = 0
    bins = 0
    t0 = time.perf_counter()
    with threadpool_limits(1):
        while time.perf_counter() - t0 < budget:
            b = (wid + n) % mix.shape[0]
            O.oracle_debug_loop(mix[b], tgt[b], itf[b], n_fft=N_FFT, hop=HOP, sigma=1.0)
            bins += (N_FFT // 2 + 1) * O.n_frames(mix.shape[-1], N_FFT, HOP)
            n += 1
    return n, bins, time.perf_counter() - t0


def cpu_baseline(sample, seconds, workers):
    """The loop-faithful oracle_debug restatement (oracle/avz_oracle.py, kind 'port')
    on the host cores, time-boxed, one single-threaded worker process per core."""
    import multiprocessing as mp
    global _CPU_SAMPLE
    _CPU_SAMPLE = sample
    ctx = mp.get_context("fork")  # forked before any GPU initialisation
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(w, seconds) for w in range(workers)])
    wall = time.perf_counter() - t0
    utts = sum(r[0] for r in res)
    bins = sum(r[1] for r in res)
    return {"value": bins / max(r[2] for r in res), "unit": "TF-bins/s", "cores": workers,
            "kind": "port",
            "sample": (f"time-boxed {seconds:.0f} s x {workers} single-threaded workers over "
                       f"{sample[0].shape[0]} distinct configs[1] utterances (4.0 s, 1024/512, "
                       f"oracle IBM, sigma 1): {utts} utterances; loop-faithful restatement of "
                       f"oracle_debug.main minus WAV I/O; wall {wall:.1f} s")}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    S = int(SECONDS * FS)
    B = args.batch

    from avz import synth
    mix, tgt, itf = synth.make_batch(B, start=rank * B, n_samples=S,
                                     n_interferers=args.interferers)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        workers = args.cpu_workers or min(16, len(os.sched_getaffinity(0)))
        k = min(B, 32)
        cpu = cpu_baseline((mix[:k], tgt[:k], itf[:k]), args.cpu_seconds, workers)

    import torch
    import torch.distributed as dist

    import avz
    from avz import metrics
    from oracle import avz_oracle as O

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    plan = avz.MVDRPlan(n_fft=N_FFT, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=B, max_samples=S)
    d_mix = torch.from_numpy(mix).to(dev)
    d_tgt = torch.from_numpy(tgt).to(dev)
    d_itf = torch.from_numpy(itf).to(dev)
    lens = torch.full((B,), S, dtype=torch.int32, device=dev)
    out = plan.alloc_out(B, S, dev)
    peak = torch.empty((B,), dtype=torch.float32, device=dev)

    def step():
        plan.run(d_mix, lens, max_len=S, ref_tgt=d_tgt, ref_int=d_itf, out=out, peak=peak)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    K = args.steps
    if not args.no_kernel_timing:
        plan.set_timing(True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record()
        step()
        ev[i][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    chain_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    kt = plan.timing() if not args.no_kernel_timing else None

    # ---- final metrics: projection SIR per utterance (run_metrics.py:6-36), RCCL all-reduce
    n_out = plan.out_len(S)
    L = min(n_out, S)
    # run_metrics.calculate_metrics_manual SIR of output and of mic 1, on the device
    # (avz_projection_metrics), one call for both
    est = torch.cat([out[:, :L], d_mix[:, 0, :L]])
    m = metrics.projection_metrics(est, torch.cat([d_tgt[:, :L]] * 2),
                                   torch.cat([d_itf[:, :L]] * 2))
    sir_out, sir_in = m[:B, 3], m[B:, 3]
    sums = torch.stack([sir_in.sum(), sir_out.sum(), torch.tensor(float(B), device=dev,
                                                                  dtype=torch.float64)])
    if world > 1:
        dist.all_reduce(sums)
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        mx = torch.tensor([chain_ms] + ([kt[k] for k in plan.KERNELS] if kt else []),
                          dtype=torch.float64, device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        chain_ms = float(mx[0])
        if kt:
            kt.update({k: float(mx[1 + j]) for j, k in enumerate(plan.KERNELS)})
    # SIR delta vs the reference restatement on identical inputs (rank 0, few utterances)
    d_sir = None
    if rank == 0:
        k = min(B, 4)
        got = sir_out[:k].cpu().numpy()
        refs = []
        for b in range(k):
            r = O.oracle_debug_vec(mix[b], tgt[b], itf[b], n_fft=N_FFT, hop=HOP, sigma=1.0)
            refs.append(O.projection_sdr_sir(r[:L], tgt[b, :L], itf[b, :L])[1])
        d_sir = float(np.max(np.abs(got - np.array(refs))))

    t_max = float(elapsed.item())
    F, T = N_FFT // 2 + 1, -(-S // HOP) + 1
    bins_per_rank = B * F * T
    value = world * bins_per_rank * K / t_max
    # Algorithmic bytes: the analysis kernel reads the 2 mic + 2 reference
    # streams (4 x 4 B per sample = 15.97 B per TF-bin); the whole chain adds the output
    # stream (19.96 B per TF-bin).
    alg_analysis = B * 4 * S * 4
    alg_chain = B * (4 * S * 4 + n_out * 4)
    traffic = {}
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        pm = json.load(open(tf))
        if pm.get("batch") == B and pm.get("n_fft") == N_FFT and pm.get("samples") == S:
            traffic = pm.get("hbm_bytes_per_launch", {})
            if not isinstance(traffic, dict):
                traffic = {}
    if kt:
        dom_ms = kt["analysis"]
        roof = {"bound": "hbm", "achieved": alg_analysis / (dom_ms * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": alg_analysis / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "traffic": traffic.get("analysis"),
                "kernel": "avz_analysis_kernel<1024,IBM>", "kernel_ms": dom_ms,
                "alg_bytes_per_launch": alg_analysis,
                "kernels_ms": {k: kt[k] for k in plan.KERNELS},
                "chain": {"achieved": alg_chain / (chain_ms * 1e-3) / 1e9, "ms": chain_ms,
                          "alg_bytes_per_launch": alg_chain,
                          "frac": alg_chain / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "traffic": traffic.get("chain")}}
    else:
        roof = {"bound": "hbm", "achieved": alg_chain / (chain_ms * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": alg_chain / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "traffic": traffic.get("chain"), "kernel": "avz_mvdr_batch chain",
                "kernel_ms": chain_ms, "alg_bytes_per_launch": alg_chain}
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "TF-bins/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": 1e3 * t_max / K,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic speech-like 2-mic far-field mixtures (SURVEY 8(d)), seeds 1000+idx",
            "config": {"workload": "configs[1]: B=256 utterances/GPU, 2 interferers, oracle IBM, "
                                   "1024-pt STFT hop 512 @16 kHz, 4.0 s utterances",
                       "batch_per_gpu": B, "global_batch": B * world, "samples": S,
                       "n_fft": N_FFT, "hop": HOP, "tf_bins_per_utt": F * T, "sigma": 1.0,
                       "mask": "ibm", "postfilter": "ibm", "normalize": "peak",
                       "parallelism": f"utterance-sharded x{world}, RCCL metric all-reduce only"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "sir": {"sir_in_mean_db": float(sums[0] / sums[2]),
                    "sir_out_mean_db": float(sums[1] / sums[2]),
                    "sir_abs_delta_vs_reference_db": d_sir, "n_utts": int(sums[2])},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
