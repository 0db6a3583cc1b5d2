#!/bin/bash
# GPU session B: multi-stream graph per-client step (test + ResNet-18 preset bench).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_gpu.py -k "multistream or hip_graph" -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_seqgraph.log 2>&1 || { tail -40 gpurun_out/pt_seqgraph.log; exit 1; }
tail -4 gpurun_out/pt_seqgraph.log
timeout -k 10 400 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_resnet18_cifar10_10.log 2>&1 || { tail -30 gpurun_out/bench_resnet18_cifar10_10.log; exit 1; }
tail -1 gpurun_out/bench_resnet18_cifar10_10.log
