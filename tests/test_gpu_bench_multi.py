"""bench.py's N > 1 path on the GPU box: two fresh ranks on cuda:0 over gloo
(--rehearse-shared-gpu), each running bench.main() exactly as torch.distributed.run would
start it (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* in the environment). Checks the
rank-0 JSON line against the contract (n_gpus, global batch, configs[2]'s per-GPU shard,
value = world x bins x K / t_max, no secondary block) and its metric sums against ONE
process scoring the same 1024 utterances -- the serial loop this path replaces is
Final_pipeline/batch_run.py:12-49."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

STEPS = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.argv = ["bench.py", "--gpus", str(world), "--rehearse-shared-gpu", "--no-cpu",
                "--steps", str(STEPS), "--warmup", "1", "--no-settle"]
    import bench
    with open(out_path + f".{rank}", "w") as f:
        so = sys.stdout
        sys.stdout = f
        try:
            bench.main()
        finally:
            sys.stdout = so


def _line(path):
    lines = [l for l in open(path).read().splitlines() if l.startswith("{")]
    assert len(lines) == 1, lines
    return json.loads(lines[0])


def test_bench_two_ranks_shared_gpu(tmp_path, gpu_device):
    out = str(tmp_path / "bench")
    mp.spawn(_rank, args=(2, _free_port(), out), nprocs=2, join=True)
    line = _line(out + ".0")
    assert os.path.getsize(out + ".1") == 0  # only rank 0 prints
    cfg = line["config"]
    assert line["n_gpus"] == 2 and line["steps"] == STEPS
    assert cfg["batch_per_gpu"] == 512 and cfg["global_batch"] == 2 * cfg["batch_per_gpu"]
    assert cfg["workload"].startswith("configs[2] per-GPU shard") and "3 interferers" in cfg["workload"]
    assert "secondary" not in line
    assert line["scaling"] == "weak" and line["metric"] == json.load(
        open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    bins = cfg["batch_per_gpu"] * cfg["tf_bins_per_utt"]
    t_max = line["ms_per_step"] * STEPS / 1e3
    assert line["value"] == pytest.approx(2 * bins * STEPS / t_max, rel=1e-9)
    assert line["sir"]["n_utts"] == 1024 and line["sir"]["n_ok"] == 1024

    # one process over the same 1024 utterances (batch 0 = utterances 0 .. 1023)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "1024",
                        "--interferers", "3", "--no-cpu", "--no-secondary", "--steps", "2",
                        "--warmup", "1", "--no-settle", "--no-kernel-timing"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env={k: v for k, v in os.environ.items()
                            if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr[-2000:]
    one = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert one["sir"]["n_utts"] == 1024
    for k in ("sir_in_mean_db", "sir_out_mean_db", "osinr_out_mean_db"):
        assert line["sir"][k] == pytest.approx(one["sir"][k], abs=1e-9), k
    print(f"2 ranks: {line['value'] / 1e9:.1f} G TF-bins/s on one shared GPU; "
          f"SIR out {line['sir']['sir_out_mean_db']:.4f} dB = one process's")
