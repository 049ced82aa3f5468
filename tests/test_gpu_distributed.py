"""Multi-process path on the HIP engine: two ranks share cuda:0 over gloo,
each generating its contiguous utterance shard in HBM and beamforming it with the default
avz_mvdr_batch enhancer (deferred normalisation); the all-reduced metric sums and the CSV
rows must equal one process running the whole batch. This is the code path
`bench.py --gpus N` and `avz.batch_run` take on an 8-GPU node (there with RCCL), the
reference's serial loop being Final_pipeline/batch_run.py:12-49."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_distributed import _free_port

N_RUNS = 7
START = 5
SECONDS = 1.0
BATCH = 3  # several launches per rank, the last one partial


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from avz import batch_run
    res = batch_run.run_batch(N_RUNS, start_idx=START, n_interferers=3, seconds=SECONDS,
                              batch=BATCH, device="cuda:0",
                              csv_path=os.path.join(outdir, "batch_metrics.csv"))
    np.save(os.path.join(outdir, f"sums_{rank}.npy"), res.sums)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_hip_shards_match_single_process(gpu_device, tmp_path):
    from avz import batch_run
    single = batch_run.run_batch(N_RUNS, start_idx=START, n_interferers=3, seconds=SECONDS,
                                 batch=BATCH, device=gpu_device)
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        np.testing.assert_allclose(np.load(tmp_path / f"sums_{r}.npy"), single.sums,
                                   rtol=1e-12)
    lines = (tmp_path / "batch_metrics.csv").read_text().strip().splitlines()
    assert lines[0].split(",") == batch_run.CSV_HEADER
    rows = [l.split(",") for l in lines[1:]]
    assert [r[0] for r in rows] == [f"batch_test_{i:03d}" for i in range(START, START + N_RUNS)]
    # per-utterance results do not depend on which rank or launch carried the utterance
    assert [[r["SIR_Base"], r["SIR_Enh"], r["SINR_Base"], r["SINR_Enh"]] for r in single.rows] \
        == [[r[1], r[2], r[4], r[5]] for r in rows]
    assert single.sums[4] == N_RUNS
    assert single.mean_sir_improvement > 3.0
