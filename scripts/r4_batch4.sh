#!/bin/bash
# round-4 GPU batch: correctness of the deferred BN finalisation + new kernels, then A/B benches
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py tests/test_native_resnet18_gpu.py tests/test_determinism.py tests/test_rccl_dist_gpu.py tests/test_plane_ops_gpu.py tests/test_spectral_gpu.py tests/test_batched_rnn_gpu.py tests/test_fc_head_gpu.py tests/test_recompute_y_gpu.py tests/test_fused_block_out_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t4.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench_lazy.json 2>&1" \
 "FEDML_AMD_BN_LAZY=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench_nolazy.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_lazy.json 2>&1" \
 "FEDML_AMD_BN_LAZY=0 timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_nolazy.json 2>&1" \
 "FEDML_AMD_RECOMPUTE_Y=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench_ry.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_mnet_auto.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 --client-exec sequential > gpurun_out/r4_mnet_seq.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset rnn_shakespeare_10 --steps 2 --warmup 1 > gpurun_out/r4_rnn_batched.json 2>&1" \
 "FEDML_AMD_BATCHED_RNN=0 timeout -k 10 300 python -u bench.py --preset rnn_shakespeare_10 --steps 1 --warmup 1 --samples-per-client 400 > gpurun_out/r4_rnn_seq.json 2>&1"
