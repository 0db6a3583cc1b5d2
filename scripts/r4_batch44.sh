#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b44
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_native_resnet_fp32_gpu.py -m gpu -x -q -k 'conv3x3 or step_f32' --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/b44/tests.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b44/h.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b44/c13.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b44/r18f.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b44/h2.json 2>&1"
