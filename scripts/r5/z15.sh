#!/bin/bash
# round 5, call Z15: final rocprofv3 kernel statistics of the headline and of ResNet-18 bf16 / fp32
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z15
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
R=$PWD
prof() { local tag=$1; shift; cd /tmp; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z15/$tag -o run --output-format csv -- python3 $R/bench.py "$@" > $R/gpurun_out/r5z15/$tag.log 2>&1; local rc=$?; cd $R; f=$(find gpurun_out/r5z15/$tag -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/r5z15/${tag}_summary.txt 2>&1; find gpurun_out/r5z15/$tag -name '*kernel_trace.csv' -delete; return $rc; }
prof headline --steps 3 --warmup 1 && prof r18_bf16 --preset resnet18_cifar10_10 --dtype bf16 --steps 1 --warmup 1 && prof r18_fp32 --preset resnet18_cifar10_10 --dtype fp32 --steps 1 --warmup 1
