#!/bin/bash
# GPU session E: transformer kernels (bf16 weight shadow) + transformer presets + kernel stats.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_tf.log 2>&1 || { tail -40 gpurun_out/pt_tf.log; exit 1; }
tail -1 gpurun_out/pt_tf.log
for p in vit_b16_32 distilbert_fedopt_32; do
  timeout -k 10 500 python -u bench.py --preset $p --steps 2 --warmup 1 > gpurun_out/bench_$p.log 2>&1 || { tail -30 gpurun_out/bench_$p.log; exit 1; }
  tail -1 gpurun_out/bench_$p.log | cut -c1-160
done
PRESETS=vit_b16_32 bash scripts/gpu_prof_tf.sh
