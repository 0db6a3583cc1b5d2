#!/bin/bash
# round 5, call Z5: 64-channel 3x3 tile-kernel unit size / workgroup count sweep on ResNet-18 bf16
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z5
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
B="python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16"
run() { local tag=$1; shift; env "$@" timeout -k 10 300 $B > gpurun_out/r5z5/$tag.txt 2>&1; local rc=$?; tail -1 gpurun_out/r5z5/$tag.txt | cut -c1-120 | sed "s/^/$tag /"; return $rc; }
run base X=1 && run px256 FEDML_AMD_C3_PX64=256 && run px512 FEDML_AMD_C3_PX64=512 && run wgs1024 FEDML_AMD_C3G_WGS=1024 && run wgs4096 FEDML_AMD_C3G_WGS=4096 && run px256w1024 FEDML_AMD_C3_PX64=256 FEDML_AMD_C3G_WGS=1024
