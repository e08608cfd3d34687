#!/bin/bash
# Solo rounds: live moves above which a round goes to the grid (S2LC_SOLO_MAXLIVE)
# vs the C5-class timings (from the repo root, via gpurun):  bash tools/maxlive_sweep.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:-mls}
mkdir -p "$OUT"
for rep in 1 2; do
  for m in ${MLS:-8 16 32 64 100000}; do
    S2LC_SOLO_MAXLIVE=$m timeout -k 10 120 python3 tools/c5run.py C5 C5wide H174 > "$OUT/m$m.$rep.jsonl" 2> "$OUT/m$m.$rep.err" || exit $?
    echo "$rep maxlive=$m $(python3 -c "import json; print([(d['name'], d['warm_s'], round(d['level_solo_ms'],1), d['level_solo_rounds']) for d in map(json.loads, open('$OUT/m$m.$rep.jsonl'))])")"
  done
done
