#!/bin/bash
# Round 3, batch m: config 5 on the device data plane with per-silo slot allocations (fp32, bf16, 2 procs/silo).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_device_mailbox_gpu.py -m gpu \
  > gpurun_out/t_m.log 2>&1; rc=$?; tail -2 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
echo "== probe"; timeout -k 10 150 python -u scripts/ipc_probe.py --mode torch --children 8 --P 43000000 --child-timeout 60 > gpurun_out/ipc_probe.log 2>&1
grep '^{' gpurun_out/ipc_probe.log | tr '\n' ' ' | cut -c1-400; echo
hier() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u scripts/bench_hier.py --timeout $((t - 20)) "$@" > gpurun_out/hier_$n.log 2>&1; local rc=$?
  grep '^{' gpurun_out/hier_$n.log | cut -c1-330; grep "complete in\|opened in" gpurun_out/hier_$n.log | cut -c60-160 | tail -6
  [ $rc -eq 0 ] || { grep -v "INFO" gpurun_out/hier_$n.log | tail -40; exit $rc; }
}
hier dev_fp32 300 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device
hier dev_bf16 300 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --silo-transport device --dtype bf16
hier pps2_dev 300 --silos 4 --local-clients 4 --procs-per-silo 2 --rounds 3 --warmup 1 --silo-transport device
