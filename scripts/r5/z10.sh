#!/bin/bash
# round 5, call Z10: row-path tile loader of the 3x3 kernels: tests + benches
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z10
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z10/$tag.txt 2>&1; local rc=$?; tail -1 gpurun_out/r5z10/$tag.txt | cut -c1-110 | sed "s/^/$tag /"; return $rc; }
timeout -k 10 600 $T tests/test_native_resnet_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet18_gpu.py tests/test_native_graph_lazy_gpu.py > gpurun_out/r5z10/tests.txt 2>&1; rc=$?; tail -1 gpurun_out/r5z10/tests.txt
[ $rc -eq 0 ] || exit $rc
R18="timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1"
run r18_bf16 X=1 $R18 --dtype bf16 && run r18_fp32 X=1 $R18 --dtype fp32 && run hl X=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 && run c13 X=1 timeout -k 10 300 python -u bench.py --clients 13 --steps 40 --warmup 5
