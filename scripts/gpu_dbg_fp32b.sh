#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_default.txt 2>&1 || exit 1
FEDML_AMD_C1_FUSED=0 timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_noc1f.txt 2>&1 || exit 1
FEDML_AMD_CONV3X3=0 timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_noc3.txt 2>&1 || exit 1
FEDML_AMD_CONV3X3=0 FEDML_AMD_C1_FUSED=0 FEDML_AMD_CONV1X1=0 timeout -k 10 120 python scripts/dbg_fp32_step.py > gpurun_out/dbg_generic.txt 2>&1 || exit 1
