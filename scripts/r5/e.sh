#!/bin/bash
# round 5, call E: in-place padded Stockham FFT; cheetah vs fp64; side-stream overlap under graphs (graph queues) and eager
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5e
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 $T tests/test_spectral_gpu.py -s > gpurun_out/r5e/t_fft.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/dbg_cheetah.py 0.002 fp32 > gpurun_out/r5e/dbg_cheetah.txt 2>&1" \
 "DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5e/b13_q4.txt 2>&1" \
 "DEBUG_HIP_FORCE_GRAPH_QUEUES=4 FEDML_AMD_SIDE_WGRAD=0 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5e/b13_q4_noside.txt 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5e/b13_eager_side.txt 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 FEDML_AMD_SIDE_WGRAD=0 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5e/b13_eager_noside.txt 2>&1"
