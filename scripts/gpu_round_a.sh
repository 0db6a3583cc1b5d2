#!/bin/bash
# GPU session A: transformer kernel tests (incl. client-batched GEMM), DistilBERT preset, ResNet-18 plans.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_tf.log 2>&1 || { tail -30 gpurun_out/pt_tf.log; exit 1; }
tail -3 gpurun_out/pt_tf.log
timeout -k 10 400 python -u bench.py --preset distilbert_fedopt_32 --steps 2 --warmup 1 > gpurun_out/bench_distilbert_fedopt_32.log 2>&1 || { tail -30 gpurun_out/bench_distilbert_fedopt_32.log; exit 1; }
tail -1 gpurun_out/bench_distilbert_fedopt_32.log
PYTHONPATH=$PWD timeout -k 10 400 python -u scripts/mb_resnet18_streams.py > gpurun_out/mb_r18s.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/mb_r18s.log; exit $rc
