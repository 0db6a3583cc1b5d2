#!/bin/bash
# det+deferred-BN diagnosis, masked-fp64 step test (both BN modes), fp32 transformer GEMM micro + counters,
# headline LDS-conflict counters after the c1f weight re-pitch, headline bench
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/diag/r4_diag3.py > gpurun_out/r4_diag3.log 2>&1" \
 "timeout -k 10 400 python -u -m pytest tests/test_native_resnet_fp32_gpu.py -k matches_reference -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t9.log 2>&1" \
 "TAG=tfg0 timeout -k 10 500 bash scripts/gpu_tfgemm_pmc.sh > gpurun_out/tfg0.log 2>&1" \
 "cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/hpmc_a -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/hpmc_a.log 2>&1 && cd $R && python3 scripts/pmc_dump.py gpurun_out/hpmc_a > gpurun_out/r4_head_lds_pmc.txt 2>&1 && rm -rf gpurun_out/hpmc_a" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_b9.json 2>&1"
