#!/bin/bash
# round 5, call Z14: bf16 3x3 weight-gradient workgroup target sweep (FEDML_AMD_C3W_WGS; default 256 for bf16)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z14
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z14/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z14/$tag.txt | cut -c1-100)" >> gpurun_out/r5z14/lines.txt; return $rc; }
B="timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16"
run base X=1 $B && run w384 FEDML_AMD_C3W_WGS=384 $B && run w512 FEDML_AMD_C3W_WGS=512 $B && run w768 FEDML_AMD_C3W_WGS=768 $B && run w1024 FEDML_AMD_C3W_WGS=1024 $B && run base2 X=1 $B && \
run hl_bf16 X=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --dtype bf16 && run hl_bf16_w512 FEDML_AMD_C3W_WGS=512 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --dtype bf16
