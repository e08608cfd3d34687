#!/bin/bash
# Packed kernel head split (S2LC_PACK_HEAD_BPC head blocks per CU running
# S2LC_PACK_HEAD_GPW groups per wave on the longest histories) vs the C4
# launch time over batch sizes (from the repo root, via gpurun):
#   bash tools/head_sweep.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:-head}
mkdir -p "$OUT"
for rep in 1 2; do
  for cfg in 0:1 1:1 1:2 2:1; do
    b=${cfg%%:*}; g=${cfg##*:}
    S2LC_PACK_HEAD_BPC=$b S2LC_PACK_HEAD_GPW=$g timeout -k 10 200 python3 tools/pack_sweep.py 1000 2500 6000 10000 \
      > "$OUT/h${b}_${g}.$rep.jsonl" 2> "$OUT/h${b}_${g}.$rep.err" || exit $?
    echo "$rep head_bpc=$b head_gpw=$g $(python3 -c "import json; print([(json.loads(l)['histories'], json.loads(l)['launch_ms']) for l in open('$OUT/h${b}_${g}.$rep.jsonl')])")"
  done
done
