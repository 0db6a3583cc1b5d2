#!/bin/bash
# rocprofv3 kernel stats of the fp32 transformer presets (template arguments kept: policy / tiles visible).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
for p in ${PRESETS:-distilbert_fedopt_32 vit_b16_32}; do
  KEEP_T=1 bash scripts/gpu_prof_preset.sh $p ${BENCH_ARGS:-} || exit 1
  head -40 gpurun_out/prof_${p}_summary.txt
done
