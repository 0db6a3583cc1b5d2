#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FEDML_AMD_POISON=1 timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_poison.txt 2>&1
FEDML_AMD_POISON=1 FEDML_AMD_CONV3X3=0 timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_poison_noc3.txt 2>&1
FEDML_AMD_POISON=1 FEDML_AMD_C1_FUSED=0 timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_poison_noc1f.txt 2>&1
