#!/bin/bash
# PMC passes over the fp32 headline (each pass its own run; --kernel-trace only with --pmc):
#   A: FETCH_SIZE + LDS bank conflicts + GRBM_GUI_ACTIVE    B: WRITE_SIZE + MFMA busy + GRBM_GUI_ACTIVE
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
OUT=${PMC_OUT:-gpurun_out/pmc_table.txt}
mkdir -p gpurun_out
ARGS=${PMC_ARGS:---steps 1 --warmup 0}
cd /tmp && export TMPDIR=/tmp
echo "== pmcA"; timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmcA -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcA.log 2>&1 || { tail -5 $R/gpurun_out/pmcA.log; exit 1; }
echo "== pmcB"; timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmcB -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcB.log 2>&1 || { tail -5 $R/gpurun_out/pmcB.log; exit 1; }
cd $R && python3 scripts/pmc_table.py $OUT gpurun_out/pmcA gpurun_out/pmcB > gpurun_out/pmc_table.log 2>&1; rc=$?
rm -rf gpurun_out/pmcA gpurun_out/pmcB
head -25 gpurun_out/pmc_table.log; exit $rc
