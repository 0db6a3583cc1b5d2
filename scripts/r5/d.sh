#!/bin/bash
# round 5, call D: side-stream 3x3 weight gradients (tests + A/B benches), cheetah vs plain-fp32 torch, 8-rank rehearsal
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5d
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 900 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/dbg_cheetah.py 0.002 fp32 > gpurun_out/r5d/dbg_cheetah.txt 2>&1" \
 "timeout -k 10 600 $T tests/test_native_graph_lazy_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_cheetah_gpu.py > gpurun_out/r5d/t_side.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py > gpurun_out/r5d/bench_side.txt 2>&1" \
 "FEDML_AMD_SIDE_WGRAD=0 timeout -k 10 300 python -u bench.py > gpurun_out/r5d/bench_noside.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5d/bench13_side.txt 2>&1" \
 "FEDML_AMD_SIDE_WGRAD=0 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5d/bench13_noside.txt 2>&1" \
 "timeout -k 10 1000 $T tests/test_rccl_dist_gpu.py -k eight > gpurun_out/r5d/t_8rank.txt 2>&1"
