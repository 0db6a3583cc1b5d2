#!/bin/bash
# round 5, call Z2: wide-conv microbench (ResNet-18 shapes, bf16) + two counter passes over it
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
R=$PWD
timeout -k 10 200 python -u scripts/mb_convk.py bf16 > gpurun_out/r5z2/mb.txt 2>&1 || exit $?
cd /tmp
pass() {
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace -d $R/gpurun_out/r5z2/p_$n -o run --output-format csv \
    -- python3 $R/scripts/mb_convk.py bf16 > $R/gpurun_out/r5z2/p_$n.log 2>&1 || { tail -5 $R/gpurun_out/r5z2/p_$n.log; exit 1; }
}
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass c TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
cd $R && python3 scripts/pmc_dump.py gpurun_out/r5z2/p_a gpurun_out/r5z2/p_b gpurun_out/r5z2/p_c > gpurun_out/r5z2/pmc_table.txt 2>&1; rc=$?
rm -rf gpurun_out/r5z2/p_a gpurun_out/r5z2/p_b gpurun_out/r5z2/p_c
exit $rc
