#!/bin/bash
# iterate: native tests → bench → (optional) profile
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
echo "== tests"; timeout -k 10 600 python -m pytest ${TESTS:-tests/test_native_resnet_gpu.py} -x -q > gpurun_out/pytest_iter.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 2 --warmup 1} > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof.log 2>&1; rc=$?
  cd $R && python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 16; exit $rc
fi
