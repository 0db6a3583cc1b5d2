#!/bin/bash
# Round 3, batch w: kernel stats of the ResNet-18 bf16 preset, round-2 tree vs this tree.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
for t in old_r2 .; do
  n=$([ $t = . ] && echo new || echo old)
  rm -rf $R/gpurun_out/prof_w_$n
  (cd /tmp && export TMPDIR=/tmp && cd $R/$t && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_w_$n -o run \
    --output-format csv -- python3 bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 1 --warmup 0 > $R/gpurun_out/prof_w_$n.log 2>&1) || exit 1
  f=$(find gpurun_out/prof_w_$n -name '*kernel_stats.csv' | head -1)
  KEEP_T=1 python3 scripts/kstats.py $f 30 > gpurun_out/prof_w_${n}_summary.txt
  find gpurun_out/prof_w_$n -name '*kernel_trace.csv' -delete
  echo "== $n"; head -22 gpurun_out/prof_w_${n}_summary.txt | cut -c1-130
done
