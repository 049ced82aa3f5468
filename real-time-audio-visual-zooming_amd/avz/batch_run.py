"""Sharded batch driver — the engine's form of Final_pipeline/batch_run.py:12-49.

The reference loops serially over run names (sim -> inf -> eval -> CSV row, exceptions
swallowed per item). Here the utterance batch is the unit of work: utterances
[start, start + n) are split contiguously over the ranks of a torch.distributed group
(one process per GPU), each rank generates its scenes ON THE DEVICE (avz_scene_generate:
counter-based draws, FFT fractional delays — milliseconds for a 512-utterance shard, so
the host never feeds the GPU), runs ONE fused MVDR launch per chunk of ``batch``
utterances, scores them on the device, and the only collective is an all-reduce of the
metric sums (RCCL over xGMI on GPUs, gloo in CPU tests; on a CPU device the scenes come
from the generator's host restatement, synth.make_batch_philox, so they are the same).

Rows follow batch_metrics.csv (Final_pipeline/src/metrics.py:16-44); STOI/PESQ are
reported as 0.0, exactly what the reference writes when pystoi/pesq are missing
(metrics.py:8-14, 148-156).
"""
from __future__ import annotations

import csv
import os
from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch
import torch.distributed as dist

from . import metrics, synth

CSV_HEADER = ["Run_ID", "SIR_Base", "SIR_Enh", "SIR_Imp", "SINR_Base", "SINR_Enh", "STOI",
              "PESQ_WB", "PESQ_NB"]


def shard(n: int, rank: int, world: int):
    """Contiguous [start, stop) of n items for this rank (sizes differ by at most one)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def allreduce_job(sums: torch.Tensor, maxes: torch.Tensor | None = None):
    """The job's only collectives: SUM of the metric sums and MAX of the
    per-rank timings (bench.py's max-over-ranks step time), in place. Every rank of a
    process group calls it -- RCCL over xGMI on GPUs, gloo in CPU tests; a one-rank group
    runs them too (identity results). No-op without a process group."""
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(sums)
        if maxes is not None:
            dist.all_reduce(maxes, op=dist.ReduceOp.MAX)
    return sums, maxes


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def finite_sums(cols, n=None):
    """SURVEY 8(e)'s metric sums with a non-finite guard, on the device: [sum of each
    column over the utterances whose every column is finite, n_ok(, n)]. One utterance with
    a NaN / inf metric (an all-zero output scores 0/0) would otherwise poison the global
    mean; the reference isolates such items per run (Final_pipeline/batch_run.py:47-49,
    its CSV row still written, metrics.py:102-123)."""
    x = torch.stack([c.double() for c in cols])
    ok = torch.isfinite(x).all(0)
    out = [torch.where(ok, x, torch.zeros_like(x)).sum(1), ok.sum().double()[None]]
    if n is not None:
        out.append(torch.full((1,), float(n), dtype=torch.float64, device=x.device))
    return torch.cat(out)


@dataclass
class BatchResult:
    rows: list            # this rank's CSV rows
    # global [sum OSIR_in, sum OSIR_out, sum OSINR_in, sum OSINR_out, n_ok, n]; the sums
    # run over the n_ok utterances whose four metrics are finite
    sums: np.ndarray

    @property
    def mean_sir_improvement(self):
        return (self.sums[1] - self.sums[0]) / max(self.sums[4], 1)


def gpu_enhancer(n_fft=1024, sigma=1.0, mic_d=0.01, max_batch=256, max_samples=64000,
                 device=None, normalize="deferred") -> Callable:
    """Returns enhance(mix[B,2,S], tgt[B,S], itf[B,S]) backed by one avz_mvdr_batch launch
    (oracle IBM, IBM post-filter) over device tensors.

    normalize="peak":     -> out[B, S_out], peak-normalised in HBM (the finalize kernel's
                          rescale pass re-reads and re-writes every sample);
    normalize="deferred": -> (out, peak): the un-normalised output and its peak; the
                          consumer applies 1 / peak (the metrics fold it into their fp64
                          sums), which skips that pass — the batch driver's default."""
    from .engine import MVDRPlan
    plan = MVDRPlan(n_fft=n_fft, sigma=sigma, mic_d=mic_d, mask="ibm", postfilter="ibm",
                    normalize="none" if normalize == "deferred" else normalize,
                    max_batch=max_batch, max_samples=max_samples)

    def enhance(mix, tgt, itf):
        out, peak = plan.run(mix, ref_tgt=tgt, ref_int=itf)
        out = out[:, :plan.out_len(mix.shape[-1])]
        return (out, peak) if normalize == "deferred" else out
    return enhance


def run_batch(n_runs: int, start_idx: int = 0, n_interferers: int = 2, *,
              seconds: float = 4.0, batch: int = 256, device=None,
              enhance: Callable | None = None, csv_path: str | None = None,
              scenes: str = "philox") -> BatchResult:
    """batch_run.run_batch equivalent over a device batch, sharded over the group.
    scenes: "philox" (device generator; host restatement on CPU) or "host" (make_batch)."""
    rank, world = world_info()
    lo, hi = shard(n_runs, rank, world)
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
        else torch.device("cpu"))
    S = int(round(seconds * synth.FS))
    if enhance is None:
        enhance = gpu_enhancer(max_batch=batch, max_samples=S, device=dev)
    rows = []
    sums = torch.zeros(6, dtype=torch.float64, device=dev)
    for c0 in range(start_idx + lo, start_idx + hi, batch):
        nb = min(batch, start_idx + hi - c0)
        if scenes == "philox" and dev.type == "cuda":
            d_mix, d_tgt, d_itf = synth.make_batch_device(nb, start=c0, n_samples=S,
                                                          n_interferers=n_interferers,
                                                          device=dev, rng="philox")
        else:
            gen = synth.make_batch_philox if scenes == "philox" else synth.make_batch
            mix, tgt, itf = gen(nb, start=c0, n_samples=S, n_interferers=n_interferers)
            d_mix = torch.from_numpy(mix).to(dev)
            d_tgt = torch.from_numpy(tgt).to(dev)
            d_itf = torch.from_numpy(itf).to(dev)
        out = enhance(d_mix, d_tgt, d_itf)
        peak = None
        if isinstance(out, tuple):  # deferred normalisation: (un-normalised out, peak)
            out, peak = out
        L = min(out.shape[-1], S)
        osinr_b, osir_b = metrics.calculate_osnr_osir(d_mix[:, 0, :L], d_tgt[:, :L], d_itf[:, :L])
        osinr_s, osir_s = metrics.calculate_osnr_osir(out[:, :L], d_tgt[:, :L], d_itf[:, :L],
                                                      peak=peak)
        sums += finite_sums([osir_b, osir_s, osinr_b, osinr_s], nb)
        vals = torch.stack([osir_b, osir_s, osinr_b, osinr_s]).cpu().numpy()
        for j in range(nb):
            rows.append({"Run_ID": f"batch_test_{c0 + j:03d}", "SIR_Base": f"{vals[0, j]:.2f}",
                         "SIR_Enh": f"{vals[1, j]:.2f}", "SIR_Imp": f"{vals[1, j] - vals[0, j]:.2f}",
                         "SINR_Base": f"{vals[2, j]:.2f}", "SINR_Enh": f"{vals[3, j]:.2f}",
                         "STOI": "0.0000", "PESQ_WB": "0.0000", "PESQ_NB": "0.0000"})
    allreduce_job(sums)  # the only collective: metric sums (+ n_ok, n)
    if csv_path is not None:
        append_csv(csv_path, rows, rank, world)
    return BatchResult(rows=rows, sums=sums.cpu().numpy())


def append_csv(path: str, rows: list, rank: int = 0, world: int = 1) -> None:
    """Concurrency-safe append: ranks write in rank order between barriers (the
    reference's header-if-absent append, metrics.py:16-44, is not safe across writers)."""
    for r in range(world):
        if r == rank:
            new = not os.path.isfile(path)
            with open(path, "a", newline="") as fh:
                w = csv.DictWriter(fh, fieldnames=CSV_HEADER)
                if new:
                    w.writeheader()
                w.writerows(rows)
        if world > 1:
            dist.barrier()
