#!/bin/bash
# Round 3, batch z: how often does the 2-rank native-engine deviation exceed the bound? (8 runs, after other tests)
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_native_resnet_gpu.py -m gpu \
  > gpurun_out/t_z0.log 2>&1; tail -1 gpurun_out/t_z0.log
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_rccl_dist_gpu.py -m gpu \
    > gpurun_out/t_z.log 2>&1
  echo "run $i: $(grep -o 'AssertionError: ([0-9.e, -]*)\|[0-9]* passed' gpurun_out/t_z.log | head -1)"
done
