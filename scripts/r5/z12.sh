#!/bin/bash
# round 5, call Z12: ResNet-18 knob sweep after the VALU-lean wide kernels (tile shape, wgrad workgroup target,
# side-stream weight gradients, C3G workgroups)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z12
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z12/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z12/$tag.txt | cut -c1-100)" >> gpurun_out/r5z12/lines.txt; return $rc; }
for dt in bf16 fp32; do
B="timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype $dt"
run ${dt}_base X=1 $B && run ${dt}_tile1 FEDML_AMD_CONVK_TILE=1 $B && run ${dt}_tile2 FEDML_AMD_CONVK_TILE=2 $B && \
run ${dt}_tile3 FEDML_AMD_CONVK_TILE=3 $B && run ${dt}_wgw512 FEDML_AMD_WGW_WGS=512 $B && run ${dt}_wgw2048 FEDML_AMD_WGW_WGS=2048 $B && \
run ${dt}_noside FEDML_AMD_SIDE_WGRAD=0 $B && run ${dt}_minK256 FEDML_AMD_CONVK_MIN_K=256 $B || exit $?
done
