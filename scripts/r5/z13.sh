#!/bin/bash
# round 5, call Z13: bf16 64-channel 3x3 tile kernel with all 64 output channels per workgroup (FEDML_AMD_C3_N64=64)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z13
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
FEDML_AMD_C3_N64=64 timeout -k 10 600 $T tests/test_native_resnet_gpu.py tests/test_native_resnet18_gpu.py > gpurun_out/r5z13/tests_n64.txt 2>&1; rc=$?; tail -1 gpurun_out/r5z13/tests_n64.txt
[ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z13/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z13/$tag.txt | cut -c1-100)" >> gpurun_out/r5z13/lines.txt; return $rc; }
B="timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16"
run base X=1 $B && run n64 FEDML_AMD_C3_N64=64 $B && run n64_px256 FEDML_AMD_C3_N64=64 FEDML_AMD_C3_PX64=256 $B && run n64_px64 FEDML_AMD_C3_N64=64 FEDML_AMD_C3_PX64=64 $B && run base2 X=1 $B && \
run hl_bf16 X=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --dtype bf16 && run hl_bf16_n64 FEDML_AMD_C3_N64=64 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --dtype bf16
