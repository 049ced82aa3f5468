"""Multi-process path on CPU (gloo, world_size 2): utterance sharding + the final
metric all-reduce give exactly the single-process result. The per-utterance enhancer
is a test stand-in built on the oracle (the GPU kernel cannot run here)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import avz_oracle as O

SECONDS = 1.0
N_RUNS = 7


def oracle_enhance(mix, tgt, itf):
    outs = [O.oracle_debug_vec(m.numpy(), t.numpy(), i.numpy(), n_fft=1024, hop=512, sigma=1.0)
            for m, t, i in zip(mix, tgt, itf)]
    return torch.from_numpy(np.stack(outs))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from avz import batch_run
    res = batch_run.run_batch(N_RUNS, start_idx=3, n_interferers=2, seconds=SECONDS, batch=2,
                              device="cpu", enhance=oracle_enhance,
                              csv_path=os.path.join(outdir, "batch_metrics.csv"))
    np.save(os.path.join(outdir, f"sums_{rank}.npy"), res.sums)
    dist.destroy_process_group()


def test_shard_covers_everything_once():
    from avz.batch_run import shard
    for n in (0, 1, 5, 7, 256, 4096):
        for world in (1, 2, 3, 8):
            spans = [shard(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and b - a >= d - c >= b - a - 1


def test_two_rank_gloo_matches_single_process(tmp_path):
    from avz import batch_run
    single = batch_run.run_batch(N_RUNS, start_idx=3, n_interferers=2, seconds=SECONDS, batch=2,
                                 device="cpu", enhance=oracle_enhance)
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        np.testing.assert_allclose(np.load(tmp_path / f"sums_{r}.npy"), single.sums, rtol=1e-12)
    lines = (tmp_path / "batch_metrics.csv").read_text().strip().splitlines()
    assert lines[0].split(",") == batch_run.CSV_HEADER
    ids = [l.split(",")[0] for l in lines[1:]]
    assert ids == [f"batch_test_{i:03d}" for i in range(3, 3 + N_RUNS)]
    assert [r["SIR_Enh"] for r in single.rows] == [l.split(",")[2] for l in lines[1:]]
    assert single.sums[4] == N_RUNS
    assert single.mean_sir_improvement > 3.0  # the oracle mask really separates the scenes
