#!/bin/bash
# GPU session D: GroupNorm kernels + ViT preset.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gn_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_gn.log 2>&1 || { tail -40 gpurun_out/pt_gn.log; exit 1; }
tail -1 gpurun_out/pt_gn.log
timeout -k 10 500 python -u bench.py --preset vit_b16_32 --steps 2 --warmup 1 > gpurun_out/bench_vit_b16_32.log 2>&1 || { tail -30 gpurun_out/bench_vit_b16_32.log; exit 1; }
tail -1 gpurun_out/bench_vit_b16_32.log
