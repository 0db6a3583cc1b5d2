#!/bin/bash
# Round 3, batch e: BASELINE config 5 (hierarchical cross-silo ViT-B/16, 8 silos x 4 local clients) on one
# MI355X: device data plane fp32 / bf16, network payloads fp32 (zero-copy frames) / int8, and a
# procs_per_silo=2 rehearsal. One line per run in gpurun_out/hier_*.log.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u scripts/bench_hier.py --timeout $((t - 20)) "$@" > gpurun_out/hier_$n.log 2>&1; local rc=$?
  grep '^{' gpurun_out/hier_$n.log | cut -c1-330; [ $rc -eq 0 ] || { tail -30 gpurun_out/hier_$n.log; exit $rc; }
}
[ -z "$TESTS" ] || { timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread $TESTS \
  > gpurun_out/t_e.log 2>&1; rc=$?; tail -4 gpurun_out/t_e.log; [ $rc -eq 0 ] || exit $rc; }
run dev_fp32 420 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device
run dev_bf16 420 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device --dtype bf16
run tcp_fp32 420 --silos 8 --local-clients 4 --rounds 3 --warmup 1
run tcp_int8 420 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --wan-compression int8
run pps2_dev 420 --silos 4 --local-clients 4 --procs-per-silo 2 --rounds 3 --warmup 1 --silo-transport device
