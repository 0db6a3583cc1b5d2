#!/bin/bash
# round 5, call Z18: repeat of the 13-client share A/B (FEDML_AMD_CONVK_MIN_K 128 vs 32), alternating, 3 pairs
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z18
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z18/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z18/$tag.txt | cut -c1-100)" >> gpurun_out/r5z18/lines.txt; return $rc; }
C13="timeout -k 10 300 python -u bench.py --clients 13 --steps 40 --warmup 5"
HL="timeout -k 10 300 python -u bench.py --steps 10 --warmup 3"
run a1 X=1 $C13 && run b1 FEDML_AMD_CONVK_MIN_K=32 $C13 && run a2 X=1 $C13 && run b2 FEDML_AMD_CONVK_MIN_K=32 $C13 && \
run a3 X=1 $C13 && run b3 FEDML_AMD_CONVK_MIN_K=32 $C13 && run ha X=1 $HL && run hb FEDML_AMD_CONVK_MIN_K=32 $HL
