#!/bin/bash
# round 5, call K: FFT occupancy fix, GN step kernel stats (no MIOpen convs), ResNet-18 benches
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5k
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 $T tests/test_spectral_gpu.py -s > gpurun_out/r5k/t_fft.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5k/pgn -o run --output-format csv -- python3 $R/bench.py --preset resnet18_gn_fed_cifar100_10 --steps 5 --warmup 2 > $R/gpurun_out/r5k/pgn.log 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r5k/r18_fp32.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 2 --warmup 1 > gpurun_out/r5k/r18_bf16.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r5k/mobilenet.txt 2>&1"
