#!/bin/bash
# round 5, call Z19: FEDML_AMD_CONVK_MIN_K default 32 — tests + the conv presets
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z19
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
( while true; do date > gpurun_out/r5z19/heartbeat; sleep 30; done ) &
HB=$!
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_native_resnet_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet18_gpu.py tests/test_native_graph_lazy_gpu.py tests/test_rccl_dist_gpu.py tests/test_model_zoo_gpu.py tests/test_plane_ops_gpu.py tests/test_native_resnet_gn_gpu.py > gpurun_out/r5z19/tests.txt 2>&1; rc=$?; tail -1 gpurun_out/r5z19/tests.txt
[ $rc -eq 0 ] || { kill $HB; exit $rc; }
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z19/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z19/$tag.txt | cut -c1-100)" >> gpurun_out/r5z19/lines.txt; return $rc; }
B="timeout -k 10 300 python -u bench.py"
run r18_bf16 X=1 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16 && run r18_bf16_128 FEDML_AMD_CONVK_MIN_K=128 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype bf16 && \
run r18_fp32 X=1 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype fp32 && run r18_fp32_128 FEDML_AMD_CONVK_MIN_K=128 $B --preset resnet18_cifar10_10 --steps 3 --warmup 1 --dtype fp32 && \
run mobilenet X=1 $B --preset mobilenet_cifar10_10 --steps 2 --warmup 1 && run mobilenet_128 FEDML_AMD_CONVK_MIN_K=128 $B --preset mobilenet_cifar10_10 --steps 2 --warmup 1 && \
run gn X=1 $B --preset resnet18_gn_fed_cifar100_10 --steps 5 --warmup 2 && run gn_128 FEDML_AMD_CONVK_MIN_K=128 $B --preset resnet18_gn_fed_cifar100_10 --steps 5 --warmup 2 && \
run hl X=1 $B --steps 10 --warmup 3 && run c13 X=1 $B --clients 13 --steps 40 --warmup 5
rc=$?
kill $HB
exit $rc
