#!/bin/bash
# round 5, call Z22: transposed-LDS fragments built as one 8-lane vector (no v_bfi per fragment): bf16 benches,
# then the whole GPU suite + smoke
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z22
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z22/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z22/$tag.txt | cut -c1-100)" >> gpurun_out/r5z22/lines.txt; return $rc; }
B="timeout -k 10 300 python -u bench.py"
run r18_bf16 X=1 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16 && \
run vit_bf16 X=1 $B --preset vit_b16_32 --steps 3 --warmup 1 --dtype bf16 && \
run distilbert_bf16 X=1 $B --preset distilbert_fedopt_32 --steps 3 --warmup 1 --dtype bf16 && \
run hl_bf16 X=1 $B --steps 5 --warmup 2 --dtype bf16 && run hl X=1 $B --steps 10 --warmup 3 || exit $?
bash scripts/r5/full.sh
