#!/bin/bash
# c1f swizzled LDS layouts: numerics + headline bench + LDS counters; config 5 with 2 processes per silo
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_recompute_y_gpu.py tests/test_fused_block_out_gpu.py tests/test_bconv_native_gpu.py tests/test_native_resnet18_gpu.py tests/test_plane_ops_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t11.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_swz.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/r4_c13_swz.json 2>&1" \
 "cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/hpmc_b -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/hpmc_b.log 2>&1 && cd $R && python3 scripts/pmc_dump.py gpurun_out/hpmc_b > gpurun_out/r4_head_lds_pmc_swz.txt 2>&1 && rm -rf gpurun_out/hpmc_b" \
 "timeout -k 10 700 python -u scripts/bench_hier.py --silos 8 --local-clients 4 --procs-per-silo 2 --server-cpu --rounds 1 --warmup 1 --timeout 660 > gpurun_out/r4_hier_8x4_pps2.log 2>&1"
