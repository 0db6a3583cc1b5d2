#!/bin/bash
# round 6, call B12: counter passes over the headline step with the c1x kernels (MFMA busy, waits, LDS conflicts,
# VALU per MFMA) — scripts/layer_prof.py --C 100, profiled kernels serialised
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b12 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
R=$PWD
cd /tmp
export FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0
bash $R/scripts/gpu_steps.sh \
 "timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/p1 -o run -- python3 $R/scripts/layer_prof.py --model resnet56 --C 100 --N 64 --dtype fp32 --steps 2 > $R/$O/p1.txt 2>&1" \
 "timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/p2 -o run -- python3 $R/scripts/layer_prof.py --model resnet56 --C 100 --N 64 --dtype fp32 --steps 2 > $R/$O/p2.txt 2>&1"
rc=$?
cd $R
kill $HB
python3 scripts/pmc_dump.py $O/p1 $O/p2 > $O/pmc.txt 2>&1; grep -A4 'c1x' $O/pmc.txt | grep -E 'c1x|->' | cut -c1-200
exit $rc
