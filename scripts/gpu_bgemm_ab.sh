#!/bin/bash
# A/B of the client-batched GEMM LDS schemes (FEDML_AMD_BGEMM_DB=1 double buffer / 0 single buffer,
# 3 blocks per CU): kernel tests, microbench, ViT preset.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_tf.log 2>&1 || { tail -30 gpurun_out/pt_tf.log; exit 1; }
tail -1 gpurun_out/pt_tf.log
for db in 1 0; do
  echo "== DB=$db"
  FEDML_AMD_BGEMM_DB=$db PYTHONPATH=$PWD timeout -k 10 300 python -u scripts/mb_bgemm.py > gpurun_out/mb_bgemm_db$db.log 2>&1 || { tail -20 gpurun_out/mb_bgemm_db$db.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/mb_bgemm_db$db.log
done
timeout -k 10 500 python -u bench.py --preset vit_b16_32 --steps 2 --warmup 1 > gpurun_out/bench_vit_b16_32.log 2>&1 || { tail -30 gpurun_out/bench_vit_b16_32.log; exit 1; }
tail -1 gpurun_out/bench_vit_b16_32.log | cut -c1-130
