#!/bin/bash
# the C4 line only, a few runs (diagnostics)
set -uo pipefail
OUT=gpurun_out/${1:-bq}
mkdir -p "$OUT"
for k in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-c5 --no-small --no-e2e --steps 20 > "$OUT/b$k.json" 2> "$OUT/b$k.err" || exit $?
  python3 -c "import json; d=json.load(open('$OUT/b$k.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['kernel_ms'])"
done
