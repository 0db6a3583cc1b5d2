#!/bin/bash
# round 5, call B: native inference + GN step + radix-8 FFT tests, re-runs, S-FedAvg bench, GN bench, kernel traces
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5b
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 $T tests/test_native_resnet_gn_gpu.py tests/test_spectral_gpu.py -s > gpurun_out/r5b/t_gn_fft.txt 2>&1" \
 "timeout -k 10 600 $T tests/test_valued_rccl_gpu.py tests/test_native_graph_lazy_gpu.py tests/test_cheetah_gpu.py tests/test_fed_plane.py > gpurun_out/r5b/t_rerun.txt 2>&1" \
 "timeout -k 10 600 $T tests/test_model_zoo_gpu.py -k 'fp32 and (rnn or mobilenet_v3 or efficientnet or resnet18_gn)' > gpurun_out/r5b/t_zoo.txt 2>&1" \
 "timeout -k 10 500 python -u scripts/bench_valued.py --rounds 2 > gpurun_out/r5b/bench_valued.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_gn_fed_cifar100_10 --steps 10 --warmup 3 > gpurun_out/r5b/bench_gn.txt 2>&1" \
 "FEDML_AMD_NATIVE_CONV=0 timeout -k 10 300 python -u bench.py --preset resnet18_gn_fed_cifar100_10 --steps 10 --warmup 3 > gpurun_out/r5b/bench_gn_seq.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5b/p13 -o run --output-format csv -- python3 $R/bench.py --clients 13 --steps 3 --warmup 1 > $R/gpurun_out/r5b/p13.log 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5b/p100 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/r5b/p100.log 2>&1"
