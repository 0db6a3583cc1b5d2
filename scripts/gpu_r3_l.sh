#!/bin/bash
# Round 3, batch l: BASELINE config 5 over the network transport (fp32 state dicts, int8 WAN), bf16, then the HIP-IPC
# import probe (why the device plane stalls with 8 silo processes).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
hier() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u scripts/bench_hier.py --timeout $((t - 20)) "$@" > gpurun_out/hier_$n.log 2>&1; local rc=$?
  grep '^{' gpurun_out/hier_$n.log | cut -c1-330; grep "complete in" gpurun_out/hier_$n.log | cut -c60-160 | tail -5
  [ $rc -eq 0 ] || { grep -v "INFO" gpurun_out/hier_$n.log | tail -40; exit $rc; }
}
hier tcp_fp32 300 --silos 8 --local-clients 4 --rounds 3 --warmup 1
hier tcp_int8 300 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --wan-compression int8
hier tcp_bf16 300 --silos 8 --local-clients 4 --rounds 3 --warmup 1 --dtype bf16
for m in "--mode torch --children 2" "--mode torch --children 8" "--mode torch --children 8 --serial" "--mode raw --children 8"; do
  echo "== probe $m"; timeout -k 10 150 python -u scripts/ipc_probe.py $m --child-timeout 60 > gpurun_out/ipc_probe.log 2>&1; rc=$?
  grep '^{' gpurun_out/ipc_probe.log | tr '\n' ' ' | cut -c1-600; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/ipc_probe.log; exit $rc; }
done
hier pps2_tcp 300 --silos 4 --local-clients 4 --procs-per-silo 2 --rounds 3 --warmup 1
