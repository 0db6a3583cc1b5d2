#!/bin/bash
# round 5, call B: native inference test, S-FedAvg bench with native valuation, headline/C=13 kernel traces
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5b
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 $T tests/test_valued_rccl_gpu.py > gpurun_out/r5b/t_valued.txt 2>&1" \
 "timeout -k 10 500 python -u scripts/bench_valued.py --rounds 2 > gpurun_out/r5b/bench_valued.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5b/p13 -o run --output-format csv -- python3 $R/bench.py --clients 13 --steps 3 --warmup 1 > $R/gpurun_out/r5b/p13.log 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5b/p100 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/r5b/p100.log 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 13 --N 64 --dtype fp32 --steps 2 > gpurun_out/r5b/lp13.txt 2>&1"
