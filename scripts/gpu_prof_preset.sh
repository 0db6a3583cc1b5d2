#!/bin/bash
# rocprofv3 kernel stats of one bench preset: scripts/gpu_prof_preset.sh <preset> [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
P=$1; shift
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$P -o run --output-format csv -- python3 $R/bench.py --preset $P --steps 2 --warmup 1 "$@" > $R/gpurun_out/prof_$P.log 2>&1 || exit 1
cd $R
f=$(find gpurun_out/prof_$P -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py $f 30 > gpurun_out/prof_${P}_summary.txt
find gpurun_out/prof_$P -name '*kernel_trace.csv' -delete
grep '^{' gpurun_out/prof_$P.log | cut -c1-200
