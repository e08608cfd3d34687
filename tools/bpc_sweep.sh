#!/bin/bash
# packed launch vs grid blocks per CU (S2LC_PACK_BPC; unset: the occupancy API's answer)
set -uo pipefail
OUT=gpurun_out/${1:-bpc}
mkdir -p "$OUT"
S2LC_STEP_TIMING=1 timeout -k 10 60 python3 tools/step_overhead.py > "$OUT/step.json" 2> "$OUT/step.err" || exit $?
tail -1 "$OUT/step.err"
for b in api 2 3 4; do
  if [ "$b" = api ]; then unset S2LC_PACK_BPC; else export S2LC_PACK_BPC=$b; fi
  timeout -k 10 120 python3 tools/pack_sweep.py 1000 10000 > "$OUT/b_$b.jsonl" 2> "$OUT/b_$b.err" || exit $?
  echo "bpc=$b $(python3 -c "import json; print([(json.loads(l)['histories'], json.loads(l)['launch_ms']) for l in open('$OUT/b_$b.jsonl')])")"
done
