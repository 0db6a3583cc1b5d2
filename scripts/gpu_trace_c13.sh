#!/bin/bash
# Kernel trace (timestamps) of the 8-GPU per-GPU share (13 clients) to measure GPU idle gaps.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/trace_c13
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_c13 -o run --output-format csv -- python3 $R/bench.py --clients ${CL:-13} --steps 1 --warmup 1 > $R/gpurun_out/trace_c13.log 2>&1 || { tail -20 $R/gpurun_out/trace_c13.log; exit 1; }
find $R/gpurun_out/trace_c13 -type f ! -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import csv, glob
f = glob.glob("/root/repo/gpurun_out/trace_c13/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# the timed round = the last half of the trace (2 rounds: warmup + timed)
n = len(ev); ev = ev[n // 2:]
busy = 0; end = ev[0][0]; gaps = 0
for s, e, _ in ev:
    if s > end: gaps += s - end
    busy += max(0, e - max(s, end)); end = max(end, e)
span = ev[-1][1] - ev[0][0]
print(f"launches {len(ev)}  span {span/1e6:.1f} ms  busy {busy/1e6:.1f} ms  idle {gaps/1e6:.1f} ms ({100*gaps/span:.1f}%)")
PY
