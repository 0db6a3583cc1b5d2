#!/bin/bash
# round 5, call C: GN native step (materialised-dy wgrad), backward-only recompute, cheetah diagnostic, GN bench, ryb A/B
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5c
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 $T tests/test_native_resnet_gn_gpu.py tests/test_recompute_y_gpu.py -s > gpurun_out/r5c/t_gn_ry.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/dbg_cheetah.py 0.002 > gpurun_out/r5c/dbg_cheetah.txt 2>&1" \
 "timeout -k 10 400 $T tests/test_model_zoo_gpu.py -k 'fp32 and resnet18_gn' > gpurun_out/r5c/t_zoo.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_gn_fed_cifar100_10 --steps 10 --warmup 3 > gpurun_out/r5c/bench_gn.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py > gpurun_out/r5c/bench_a.txt 2>&1" \
 "FEDML_AMD_RY_BWD=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5c/bench_ryb.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5c/bench13_a.txt 2>&1" \
 "FEDML_AMD_RY_BWD=1 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5c/bench13_ryb.txt 2>&1"
