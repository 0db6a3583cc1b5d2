#!/bin/bash
# Round 3, batch b: 2-rank native-engine rehearsal (test + bench line, gloo on one GPU), then rocprof of
# the fp32 transformer presets.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_rccl_dist_gpu.py \
  > gpurun_out/t_dist_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/t_dist_gpu.log; [ $rc -eq 0 ] || exit $rc
FEDML_AMD_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearse2_r3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/rehearse2_r3.log | tail -3; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r3_prof_tf.sh
