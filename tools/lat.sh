#!/bin/bash
# single-history drop-in latency: bench.py's C1-C3 leg only (s2lc_check cold /
# warm, the s2-porcupine CLI process with its phase breakdown)
set -uo pipefail
OUT=gpurun_out/${1:-lat}
mkdir -p "$OUT"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-c5 --no-e2e --steps 2 --histories 1000 > "$OUT/lat.json" 2> "$OUT/lat.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/lat.json')); print(json.dumps(d['c1_c3']))"
