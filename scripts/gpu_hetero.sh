#!/bin/bash
# heterogeneous (LDA alpha=0.5) vs IID headline throughput, fp32 and bf16, plus a kernel profile of the hetero run
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for args in "--steps 6 --warmup 2" "--partition hetero --steps 6 --warmup 2" "--dtype bf16 --partition hetero --steps 6 --warmup 2"; do
  echo "== bench $args"; timeout -k 10 400 python bench.py $args > gpurun_out/bench_h.log 2>&1; rc=$?; tail -1 gpurun_out/bench_h.log; [ $rc -eq 0 ] || exit $rc
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_het -o run --output-format csv -- python3 $R/bench.py --partition hetero --steps 1 --warmup 1 > $R/gpurun_out/prof_het.log 2>&1; rc=$?; tail -1 $R/gpurun_out/prof_het.log; exit $rc
