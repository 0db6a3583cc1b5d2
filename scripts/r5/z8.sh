#!/bin/bash
# round 5, call Z8: VALU-vs-MFMA counter pass over the headline step (ResNet-56 fp32, 100 clients)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z8
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
R=$PWD
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r5z8/p_a -o run --output-format csv -- python3 $R/scripts/layer_prof.py --model resnet56 --C 100 --N 64 --dtype fp32 --steps 2 > $R/gpurun_out/r5z8/p_a.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/r5z8/p_b -o run --output-format csv -- python3 $R/scripts/layer_prof.py --model resnet56 --C 100 --N 64 --dtype fp32 --steps 2 > $R/gpurun_out/r5z8/p_b.log 2>&1 || exit $?
cd $R
python3 scripts/pmc_dump.py gpurun_out/r5z8/p_a gpurun_out/r5z8/p_b > gpurun_out/r5z8/pmc_table.txt 2>&1
rm -rf gpurun_out/r5z8/p_a gpurun_out/r5z8/p_b
