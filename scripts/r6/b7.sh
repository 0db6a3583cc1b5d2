#!/bin/bash
# round 6, call B7: counter pass over the bf16 client GEMMs (ViT-B/16 shapes): MFMA busy, issue waits, LDS conflicts
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b7 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
R=$PWD
cd /tmp
bash $R/scripts/gpu_steps.sh \
 "timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/p1 -o run -- python3 $R/scripts/tf_gemm_micro.py --dtype bf16 --iters 2 > $R/$O/p1.txt 2>&1" \
 "timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/p2 -o run -- python3 $R/scripts/tf_gemm_micro.py --dtype bf16 --iters 2 > $R/$O/p2.txt 2>&1"
rc=$?
cd $R
[ $rc -eq 0 ] || [ $rc -eq 1 ] && bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13_a.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13_pb64.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13_b.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head_pb64.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head_a.txt 2>&1"
for f in c13_a c13_pb64 c13_b head_pb64 head_a; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-130)"; done
kill $HB
python3 scripts/pmc_dump.py $O/p1 $O/p2 > $O/pmc.txt 2>&1; head -40 $O/pmc.txt | cut -c1-250
exit $rc
