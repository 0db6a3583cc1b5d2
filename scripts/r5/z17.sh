#!/bin/bash
# round 5, call Z17: headline / 13-client share with more layers on the (now VALU-lean) K-streamed kernel
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z17
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z17/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z17/$tag.txt | cut -c1-100)" >> gpurun_out/r5z17/lines.txt; return $rc; }
HL="timeout -k 10 300 python -u bench.py --steps 6 --warmup 2"
C13="timeout -k 10 300 python -u bench.py --clients 13 --steps 30 --warmup 5"
run hl_128 X=1 $HL && run hl_64 FEDML_AMD_CONVK_MIN_K=64 $HL && run hl_32 FEDML_AMD_CONVK_MIN_K=32 $HL && \
run c13_128 X=1 $C13 && run c13_64 FEDML_AMD_CONVK_MIN_K=64 $C13 && run c13_32 FEDML_AMD_CONVK_MIN_K=32 $C13 && \
run hlbf_128 X=1 $HL --dtype bf16 && run hlbf_64 FEDML_AMD_CONVK_MIN_K=64 $HL --dtype bf16
