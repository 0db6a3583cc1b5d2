#!/bin/bash
# round 5, call Z6: XCD-aware block order of the 3x3 tile kernels (fwd/bwd-data and weight gradient):
# numerics tests, then A/B on ResNet-18 bf16, the headline and the 13-client share
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z6
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
( while true; do date > gpurun_out/r5z6/heartbeat; sleep 30; done ) &
HB=$!
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z6/$tag.txt 2>&1; local rc=$?; tail -1 gpurun_out/r5z6/$tag.txt | cut -c1-110 | sed "s/^/$tag /"; return $rc; }
R18="timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16"
HL="timeout -k 10 300 python -u bench.py --steps 10 --warmup 3"
C13="timeout -k 10 300 python -u bench.py --clients 13 --steps 40 --warmup 5"
timeout -k 10 600 $T tests/test_native_resnet_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet18_gpu.py tests/test_native_graph_lazy_gpu.py > gpurun_out/r5z6/tests.txt 2>&1; rc=$?; tail -1 gpurun_out/r5z6/tests.txt
[ $rc -eq 0 ] || { kill $HB; exit $rc; }
run r18_on X=1 $R18 && run r18_off FEDML_AMD_C3_XCD=0 $R18 && run hl_on X=1 $HL && run hl_off FEDML_AMD_C3_XCD=0 $HL && run c13_on X=1 $C13 && run c13_off FEDML_AMD_C3_XCD=0 $C13
rc=$?
kill $HB
exit $rc
