#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for e in "$@"; do echo "== $e"; env PYTHONPATH=. $e timeout -k 10 120 python scripts/mb_convk.py ${DT:-bf16} 2>&1 | grep -v amdgpu.ids; done
