#!/bin/bash
# packed-kernel variants (libraries built with different window / prefetch /
# occupancy settings) on the C4 launch: pack_sweep at 1,000 and 10,000
# histories per library (diagnostics)
set -uo pipefail
OUT=gpurun_out/${1:-vs}
shift
mkdir -p "$OUT"
for v in "$@"; do
  lib=$PWD/s2_verification_amd/$v
  S2LC_LIB=$lib timeout -k 10 120 python3 tools/pack_sweep.py 1 1000 10000 > "$OUT/$v.jsonl" 2> "$OUT/$v.err" || { echo "$v failed"; exit 1; }
  echo "$v $(python3 -c "import json; print([(json.loads(l)['histories'], json.loads(l)['launch_ms']) for l in open('$OUT/$v.jsonl')])")"
done
