#!/bin/bash
# rocprofv3 kernel trace + stats of the bench; summary copied to profiles/
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS:---steps 1 --warmup 1} > $R/gpurun_out/prof.log 2>&1; rc=$?
tail -2 $R/gpurun_out/prof.log
exit $rc
