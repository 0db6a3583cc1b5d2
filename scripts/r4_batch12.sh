#!/bin/bash
# headline / 13-client / MobileNet benches, then the full GPU suite (what the driver runs at round end)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_b12.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_b12.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_mnet_b12.json 2>&1" \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_gpu_suite_b12.log 2>&1"
