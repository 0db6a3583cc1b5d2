#!/bin/bash
# round 5, call Z3: VALU-lean wide conv kernels (uniform-tap convk gather, buffer-descriptor wgrad_wide rows,
# packed bf16 converts): numerics tests, microbench, ResNet-18 + headline benches
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z3
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
( while true; do date > gpurun_out/r5z3/heartbeat; sleep 30; done ) &
HB=$!
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1"
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 $T tests/test_native_resnet18_gpu.py tests/test_native_resnet_gpu.py tests/test_native_resnet_fp32_gpu.py > gpurun_out/r5z3/tests.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/mb_convk.py bf16 > gpurun_out/r5z3/mb.txt 2>&1" \
 "timeout -k 10 300 $B --dtype bf16 > gpurun_out/r5z3/r18_bf16.txt 2>&1" \
 "timeout -k 10 300 $B --dtype fp32 > gpurun_out/r5z3/r18_fp32.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5z3/headline.txt 2>&1"
rc=$?
kill $HB
exit $rc
