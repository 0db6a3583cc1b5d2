#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/prof_mnet
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/diag/r4_diag1.py > gpurun_out/r4_diag1c.log 2>&1" \
 "timeout -k 10 600 python -u -m pytest tests/test_plane_ops_gpu.py tests/test_determinism.py tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t7.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_split1.json 2>&1" "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_c1fpitch.json 2>&1" \
 "FEDML_AMD_STEP_SPLIT=2 timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_split2.json 2>&1" \
 "FEDML_AMD_STEP_SPLIT=3 timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_split3.json 2>&1" \
 "FEDML_AMD_STEP_SPLIT=2 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_split2.json 2>&1" \
 "timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mnet -o mnet -- python3 bench.py --preset mobilenet_cifar10_10 --samples-per-client 640 --steps 1 --warmup 1 > gpurun_out/r4_prof_mnet.log 2>&1"
