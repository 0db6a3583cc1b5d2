#!/bin/bash
# round 5, call I: DMA GEMM default (tests, micro, ViT/DistilBERT), fc-head 1024 threads, c1f partials A/B,
# cheetah bench lines, config-5 RCCL plane bench
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5i
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 $T tests/test_transformer_kernels_gpu.py tests/test_native_resnet_fp32_gpu.py -k 'linear or matches_reference' > gpurun_out/r5i/t_tf.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 --check > gpurun_out/r5i/micro_dma.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5i/vit.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 > gpurun_out/r5i/dbert.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py > gpurun_out/r5i/b100.txt 2>&1" \
 "FEDML_AMD_C1F_PART=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5i/b100_part.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5i/b13.txt 2>&1" \
 "FEDML_AMD_C1F_PART=1 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5i/b13_part.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_cheetah.py --model resnet56 --replicas 4 --batch-size 64 --samples 25600 --epochs 2 > gpurun_out/r5i/cheetah_native.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_cheetah.py --model resnet56 --replicas 1 --batch-size 64 --samples 12800 --epochs 2 --exec torch > gpurun_out/r5i/cheetah_torch.txt 2>&1" \
 "timeout -k 10 700 python -u scripts/bench_hier.py --silos 8 --local-clients 4 --silo-transport rccl --rounds 3 --warmup 1 > gpurun_out/r5i/hier_rccl.txt 2>&1"
