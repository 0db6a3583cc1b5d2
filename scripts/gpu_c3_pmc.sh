#!/bin/bash
# Counter passes over the fp32 3x3 kernels at the ResNet-56 / C=100 shapes (scripts/c3_time.py), one pass per
# counter group (--kernel-trace only), plus the list of counters this GPU offers.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
mkdir -p gpurun_out
SH=${SHAPES:-64x8x1,32x16x1,16x32x1}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1 || true
pass() {   # name counters...
  local n=$1; shift
  echo "== $n"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $R/gpurun_out/c3pmc_$n -o run --output-format csv \
    -- python3 $R/scripts/c3_time.py --iters 3 --shapes $SH > $R/gpurun_out/c3pmc_$n.log 2>&1 || { tail -5 $R/gpurun_out/c3pmc_$n.log; exit 1; }
}
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES
cd $R && python3 scripts/pmc_dump.py gpurun_out/c3pmc_a gpurun_out/c3pmc_b > gpurun_out/c3pmc_table.txt 2>&1; rc=$?
rm -rf gpurun_out/c3pmc_a gpurun_out/c3pmc_b
cat gpurun_out/c3pmc_table.txt | cut -c1-250; exit $rc
