#!/bin/bash
# round 6, call A10: counters of the fused inference kernels (variant 5) on the chunk shape — MFMA busy vs wave
# waits — and the S-FedAvg valuation round with variant 5
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a10 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "FEDML_AMD_BNECK_EVAL_VARIANT=5 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python3 scripts/fused_eval_micro.py --iters 1 > $O/pmc1.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=5 timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp > $O/valued_v5.txt 2>&1"
rc=$?
kill $HB
echo "valued_v5: $(tail -1 $O/valued_v5.txt | cut -c1-250)"
exit $rc
