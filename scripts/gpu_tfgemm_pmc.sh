#!/bin/bash
# Timing + counter passes over the fp32 transformer GEMMs at the ViT-B/16 preset's shapes
# (scripts/tf_gemm_micro.py), one pass per counter group (--kernel-trace only).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-tfg}
timeout -k 10 120 python3 -u scripts/tf_gemm_micro.py --check > gpurun_out/${TAG}_micro.jsonl 2>&1 || { tail -5 gpurun_out/${TAG}_micro.jsonl; exit 1; }
cd /tmp && export TMPDIR=/tmp
pass() {   # name counters...
  local n=$1; shift
  echo "== $n"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $R/gpurun_out/${TAG}pmc_$n -o run --output-format csv \
    -- python3 $R/scripts/tf_gemm_micro.py --iters 2 > $R/gpurun_out/${TAG}pmc_$n.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}pmc_$n.log; exit 1; }
}
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass c TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
cd $R && python3 scripts/pmc_dump.py gpurun_out/${TAG}pmc_a gpurun_out/${TAG}pmc_b gpurun_out/${TAG}pmc_c > gpurun_out/${TAG}pmc_table.txt 2>&1; rc=$?
rm -rf gpurun_out/${TAG}pmc_a gpurun_out/${TAG}pmc_b gpurun_out/${TAG}pmc_c
cut -c1-250 gpurun_out/${TAG}pmc_table.txt | grep -v "^$" ; exit $rc
