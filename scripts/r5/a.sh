#!/bin/bash
# round 5, call A: descriptor-lifetime fix, Cheetah native, S-FedAvg on the engine, RCCL plane + benches
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5a
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_native_graph_lazy_gpu.py tests/test_optimizer_state_reset.py tests/test_cheetah_gpu.py tests/test_valued_rccl_gpu.py tests/test_fed_plane.py > gpurun_out/r5a/tests.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5a/bench.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --clients 13 > gpurun_out/r5a/bench_c13.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 > gpurun_out/r5a/bench_valued.txt 2>&1"
