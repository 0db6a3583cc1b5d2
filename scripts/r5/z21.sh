#!/bin/bash
# round 5, call Z21: K-streamed conv with a null output (statistics-only forward of the recomputed-y backward):
# the recompute-y tests first (they faulted when such a call reached the K-streamed kernel), then the whole suite
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z21
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_recompute_y_gpu.py > gpurun_out/r5z21/ry.txt 2>&1; rc=$?; tail -1 gpurun_out/r5z21/ry.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/r5/full.sh
