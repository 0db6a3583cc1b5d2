#!/bin/bash
# full GPU suite + the bench lines of every preset (fp32; transformers also bf16)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 660 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_gpu_suite_b55.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_b55.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_b55.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --steps 4 --warmup 2 > gpurun_out/r4_vit_b55.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --steps 5 --warmup 2 > gpurun_out/r4_distil_b55.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/r4_vit_bf16_b55.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 5 --warmup 2 > gpurun_out/r4_distil_bf16_b55.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16_b55.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_mobilenet_b55.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_r18_fp32_b55.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset rnn_shakespeare_10 --steps 2 --warmup 1 > gpurun_out/r4_rnn_b55.json 2>&1" \
 "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > gpurun_out/r4_smoke_b55.txt 2>&1"
