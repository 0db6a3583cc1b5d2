#!/bin/bash
# Round 3, batch i: K12 spectral kernel tests, 3x3 counter passes, ResNet-18 (config 2) fp32 bench + kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_spectral_gpu.py tests/test_fused_block_out_gpu.py tests/test_recompute_y_gpu.py -m gpu \
  > gpurun_out/t_i.log 2>&1; rc=$?; tail -3 gpurun_out/t_i.log; [ $rc -eq 0 ] || exit $rc
for fb in 1 0; do
  FEDML_AMD_FUSE_BOUT=$fb timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b_head_fb$fb.log 2>&1; rc=$?
  echo "fuse_bout=$fb"; grep '^{' gpurun_out/b_head_fb$fb.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_c3_pmc.sh || exit 1
timeout -k 10 400 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b_r18_fp32.log 2>&1; rc=$?
grep '^{' gpurun_out/b_r18_fp32.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/b_r18_fp32.log; exit $rc; }
rm -rf gpurun_out/prof_r18
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r18 -o run \
  --output-format csv -- python3 $R/bench.py --preset resnet18_cifar10_10 --steps 1 --warmup 0 > $R/gpurun_out/prof_r18.log 2>&1) || exit 1
f=$(find gpurun_out/prof_r18 -name '*kernel_stats.csv' | head -1)
KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/prof_r18_summary.txt
find gpurun_out/prof_r18 -name '*kernel_trace.csv' -delete
head -25 gpurun_out/prof_r18_summary.txt | cut -c1-160
hier() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u scripts/bench_hier.py --timeout $((t - 20)) "$@" > gpurun_out/hier_$n.log 2>&1; local rc=$?
  grep '^{' gpurun_out/hier_$n.log | cut -c1-330; [ $rc -eq 0 ] || { grep -v "INFO" gpurun_out/hier_$n.log | tail -60; exit $rc; }
}
hier dev_small 300 --silos 2 --local-clients 2 --rounds 2 --warmup 1 --silo-transport device
hier dev_fp32 420 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device
