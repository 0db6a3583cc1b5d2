#!/bin/bash
# round 5, call A2: the new GPU tests (no -x: every file reports)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5a2
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 $T tests/test_native_graph_lazy_gpu.py tests/test_optimizer_state_reset.py tests/test_cheetah_gpu.py > gpurun_out/r5a2/t1.txt 2>&1" \
 "timeout -k 10 500 $T tests/test_valued_rccl_gpu.py tests/test_fed_plane.py > gpurun_out/r5a2/t2.txt 2>&1" \
 "timeout -k 10 600 $T tests/test_model_zoo_gpu.py > gpurun_out/r5a2/t3.txt 2>&1"
