#!/bin/bash
# run a pytest selection on the GPU box: scripts/gpu_t.sh <pytest args...>
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_sel.log; exit $rc
