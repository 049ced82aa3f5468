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


def test_finite_sums_skip_non_finite_rows():
    """SURVEY 8(e)'s [sums..., n_ok, n]: an utterance with a NaN / inf metric is left out
    of the sums and of n_ok, the others are summed exactly."""
    from avz.batch_run import finite_sums
    a = torch.tensor([1.0, 2.0, float("nan"), 4.0], dtype=torch.float64)
    b = torch.tensor([10.0, float("-inf"), 30.0, 40.0], dtype=torch.float64)
    s = finite_sums([a, b], 4).numpy()
    np.testing.assert_array_equal(s, [5.0, 50.0, 2.0, 4.0])
    s = finite_sums([a[:2], b[:1].repeat(2)]).numpy()  # no n: [sums, n_ok]
    np.testing.assert_array_equal(s, [3.0, 20.0, 2.0])


def test_batch_run_non_finite_utterance_keeps_row(tmp_path):
    """One utterance whose enhanced output is all zeros (metrics 0/0): its CSV row is still
    written (as the reference writes whatever numpy returns), the global sums and n_ok
    cover the other utterances only."""
    from avz import batch_run

    def enh(mix, tgt, itf):
        out = oracle_enhance(mix, tgt, itf)
        out[1] = 0.0
        return out

    res = batch_run.run_batch(4, start_idx=3, seconds=SECONDS, batch=4, device="cpu",
                              enhance=enh, csv_path=str(tmp_path / "m.csv"))
    ref = batch_run.run_batch(4, start_idx=3, seconds=SECONDS, batch=4, device="cpu",
                              enhance=oracle_enhance)
    assert res.sums[4] == 3 and res.sums[5] == 4
    assert np.all(np.isfinite(res.sums))
    assert res.rows[1]["SIR_Enh"] in ("nan", "-inf")
    assert len((tmp_path / "m.csv").read_text().strip().splitlines()) == 5
    # the three finite utterances sum to the same as the reference run minus utterance 1
    vals = np.array([[float(r[k]) for k in ("SIR_Base", "SIR_Enh")] for r in ref.rows])
    np.testing.assert_allclose(res.sums[:2], vals[[0, 2, 3]].sum(0), atol=0.02)
