#!/bin/bash
# kernel profile of one ResNet-18 preset round (DT=bf16|fp32)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DT=${DT:-bf16}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && env ${PENV:-X=1} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r18_$DT -o run --output-format csv -- python3 $R/bench.py --preset resnet18_cifar10_10 --dtype $DT --steps 1 --warmup 1 > $R/gpurun_out/prof_r18_$DT.log 2>&1; rc=$?; tail -1 $R/gpurun_out/prof_r18_$DT.log | cut -c1-200
cd $R; f=$(find gpurun_out/prof_r18_$DT -name '*kernel_stats.csv' | head -1); KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/prof_r18_${DT}_summary.txt 2>&1 || cp $f gpurun_out/prof_r18_${DT}_summary.txt
find gpurun_out/prof_r18_$DT -name '*kernel_trace.csv' -delete
head -30 gpurun_out/prof_r18_${DT}_summary.txt | cut -c1-220
exit $rc
