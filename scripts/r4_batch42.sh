#!/bin/bash
# per-step byte / FLOP budgets (layer_prof) + smoke
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b42
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 100 --N 64 --dtype fp32 --steps 2 > gpurun_out/b42/c100.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/layer_prof.py --C 13 --N 64 --dtype fp32 --steps 3 > gpurun_out/b42/c13.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype fp32 --steps 2 > gpurun_out/b42/r18f.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype bf16 --steps 2 > gpurun_out/b42/r18b.txt 2>&1" \
 "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > gpurun_out/b42/smoke.txt 2>&1"
