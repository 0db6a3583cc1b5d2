#!/bin/bash
# Round 3, batch j: BASELINE config 5 (hierarchical cross-silo ViT-B/16, 8 silos x 4 local clients) on one MI355X after
# the silo-engine reuse / sample-count / IPC-open fixes: device plane fp32 + bf16, TCP fp32 + int8, procs_per_silo=2.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_device_mailbox_gpu.py \
  tests/test_hier_silo.py -m gpu > gpurun_out/t_j.log 2>&1; rc=$?; tail -3 gpurun_out/t_j.log; [ $rc -eq 0 ] || exit $rc
hier() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u scripts/bench_hier.py --timeout $((t - 20)) "$@" > gpurun_out/hier_$n.log 2>&1; local rc=$?
  grep '^{' gpurun_out/hier_$n.log | cut -c1-330; grep "complete in\|opened in" gpurun_out/hier_$n.log | cut -c1-160 | tail -12
  [ $rc -eq 0 ] || { grep -v "INFO" gpurun_out/hier_$n.log | tail -60; exit $rc; }
}
hier dev_fp32 400 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device
hier tcp_fp32 400 --silos 8 --local-clients 4 --rounds 3 --warmup 1
hier tcp_int8 400 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --wan-compression int8
hier dev_bf16 400 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device --dtype bf16
hier pps2_dev 400 --silos 4 --local-clients 4 --procs-per-silo 2 --rounds 3 --warmup 1 --silo-transport device
