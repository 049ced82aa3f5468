#!/bin/bash
# smoke() and an N=2 rehearsal of bench.py on a one-GPU box (both ranks on cuda:0, gloo).
set -o pipefail
mkdir -p gpurun_out/mr
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/mr/smoke.log 2>&1 || { tail -20 gpurun_out/mr/smoke.log; exit 1; }
tail -2 gpurun_out/mr/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --rehearse-shared-gpu > gpurun_out/mr/n2.log 2>&1 || { tail -30 gpurun_out/mr/n2.log; exit 1; }
tail -1 gpurun_out/mr/n2.log | cut -c1-600
