#!/bin/bash
# C4 step: blocking vs polled stream wait (host overhead beside the kernel)
set -uo pipefail
OUT=gpurun_out/${1:-sync}
mkdir -p "$OUT"
for m in block spin; do
  S2LC_SYNC=$m S2LC_STEP_TIMING=1 timeout -k 10 120 python3 tools/step_overhead.py > "$OUT/$m.json" 2> "$OUT/$m.err" || exit $?
  echo "$m $(cat $OUT/$m.json) $(tail -1 $OUT/$m.err)"
done
