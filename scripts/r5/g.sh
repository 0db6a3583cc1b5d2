#!/bin/bash
# round 5, call G: batched middle-conv weight gradients (tests + A/B benches at 100 and 13 clients) + profile at C=13
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5g
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 $T tests/test_native_graph_lazy_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_recompute_y_gpu.py > gpurun_out/r5g/t_wb.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py > gpurun_out/r5g/b100.txt 2>&1" \
 "FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u bench.py > gpurun_out/r5g/b100_nob.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5g/b13.txt 2>&1" \
 "FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5g/b13_nob.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5g/p13 -o run --output-format csv -- python3 $R/bench.py --clients 13 --steps 3 --warmup 1 > $R/gpurun_out/r5g/p13.log 2>&1"
