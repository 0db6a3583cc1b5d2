#!/bin/bash
# block output fused into the next block's first conv at stage transitions too
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b53
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_fused_block_out_gpu.py tests/test_native_resnet_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_determinism.py tests/test_rccl_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/b53/tests.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b53/h.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b53/c13.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b53/h2.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --dtype bf16 > gpurun_out/b53/hb.json 2>&1"
