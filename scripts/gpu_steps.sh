#!/bin/bash
# Run GPU steps in order; a step that fails normally (rc 0/1: e.g. a failing test) lets the next one run, any
# other status (fault, abort 134, segfault 139, time limit 124/137) stops the call there.
#   bash scripts/gpu_steps.sh "timeout -k 10 600 python -m pytest ..." "timeout -k 10 200 python bench.py ..."
for c in "$@"; do
  echo "[gpu_steps] $c"
  bash -c "$c"
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[gpu_steps] rc=$rc: stopping"
    exit $rc
  fi
done
