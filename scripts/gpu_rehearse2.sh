#!/bin/bash
# Two-rank rehearsal of the multi-GPU headline path on a ONE-GPU box: both ranks share cuda:0 and the
# collectives run over gloo (RCCL needs a GPU per rank). 25 clients → C = 13 per rank, rank 1 holds a
# padding slot (the 8-GPU layout in miniature). Timing is meaningless; correctness is the point.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 FEDML_AMD_DIST_BACKEND=gloo
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --clients 25 --steps 2 --warmup 1 > gpurun_out/rehearse2.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/rehearse2.log | tail -5; exit $rc
