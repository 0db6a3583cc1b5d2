#!/bin/bash
# round 5, call Z11: same-box bench lines after the VALU-lean wide conv kernels and packed bf16 converts
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z11
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
( while true; do date > gpurun_out/r5z11/heartbeat; sleep 30; done ) &
HB=$!
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z11/$tag.txt 2>&1; local rc=$?; tail -1 gpurun_out/r5z11/$tag.txt | sed "s/^/$tag /" >> gpurun_out/r5z11/lines.txt; return $rc; }
B="timeout -k 10 400 python -u bench.py"
run headline X=1 $B --steps 20 --warmup 5 && \
run c13 X=1 $B --clients 13 --steps 40 --warmup 5 && \
run r18_fp32 X=1 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype fp32 && \
run r18_bf16 X=1 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16 && \
run mobilenet X=1 $B --preset mobilenet_cifar10_10 --steps 2 --warmup 1 && \
run r18gn X=1 $B --preset resnet18_gn_fed_cifar100_10 --steps 5 --warmup 2 && \
run vit_bf16 X=1 $B --preset vit_b16_32 --steps 3 --warmup 1 --dtype bf16 && \
run distilbert_bf16 X=1 $B --preset distilbert_fedopt_32 --steps 3 --warmup 1 --dtype bf16
rc=$?
kill $HB
exit $rc
