#!/bin/bash
# Round 3, batch k: software-pipelined generic conv kernel (pf) + >= 2 waves/SIMD 3x3 kernels (new = pf + mw2) — conv GPU tests, then the fp32 headline A/B against the
# previous library build (FEDML_AMD_LIB=libfedml_kernels_base.so), then a kernel profile of the new build.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_resnet_gpu.py \
  tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet18_gpu.py tests/test_fused_block_out_gpu.py \
  tests/test_recompute_y_gpu.py -m gpu > gpurun_out/t_k.log 2>&1; rc=$?; tail -3 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit $rc
for v in new base pf new base pf; do
  case $v in base) L=$R/fedml_amd/_native/libfedml_kernels_base.so ;; pf) L=$R/fedml_amd/_native/libfedml_kernels_pf.so ;; *) L= ;; esac
  FEDML_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b_k_$v.log 2>&1; rc=$?
  echo "$v: $(grep '^{' gpurun_out/b_k_$v.log | cut -c60-140)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/prof_head
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run \
  --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_head.log 2>&1) || exit 1
f=$(find gpurun_out/prof_head -name '*kernel_stats.csv' | head -1)
KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/prof_head_summary.txt
find gpurun_out/prof_head -name '*kernel_trace.csv' -delete
head -25 gpurun_out/prof_head_summary.txt | cut -c1-150
