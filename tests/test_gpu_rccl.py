"""The RCCL branch, executed: a fresh child process initialises the GPU
itself, joins a one-rank ``nccl`` (= RCCL) process group bound to cuda:0, runs the
sharded batch driver (avz.batch_run.run_batch, the reference's serial loop of
Final_pipeline/batch_run.py:12-49) and bench.py's reduction (allreduce_job: SUM of the
metric sums, MAX of the timings) through RCCL; the sums must equal the single-process
run's. A one-GPU box cannot host more ranks of a real RCCL group; the N-rank data path is
test_gpu_distributed.py (gloo, ranks sharing cuda:0) and test_distributed.py (CPU)."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_distributed import _free_port

N_RUNS = 5
START = 11
SECONDS = 1.0


def _child(rank, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from avz import batch_run
    res = batch_run.run_batch(N_RUNS, start_idx=START, n_interferers=2, seconds=SECONDS,
                              batch=2, device="cuda:0")
    sums = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    maxes = torch.tensor([0.25, 7.0], dtype=torch.float64, device=dev)
    batch_run.allreduce_job(sums, maxes)
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, "sums.npy"), res.sums)
    np.save(os.path.join(outdir, "bench_reduce.npy"), torch.cat([sums, maxes]).cpu().numpy())
    with open(os.path.join(outdir, "backend.txt"), "w") as fh:
        fh.write(str(dist.get_backend()))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_one_rank_group_matches_single_process(gpu_device, tmp_path):
    from avz import batch_run
    single = batch_run.run_batch(N_RUNS, start_idx=START, n_interferers=2, seconds=SECONDS,
                                 batch=2, device=gpu_device)
    mp.spawn(_child, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    assert (tmp_path / "backend.txt").read_text() == "nccl"
    np.testing.assert_allclose(np.load(tmp_path / "sums.npy"), single.sums, rtol=1e-12)
    np.testing.assert_array_equal(np.load(tmp_path / "bench_reduce.npy"), [1.5, 2.5, 0.25, 7.0])
    assert single.sums[4] == N_RUNS
