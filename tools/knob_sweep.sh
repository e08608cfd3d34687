#!/bin/bash
# Level-search knobs on the C5-class histories (from the repo root, via gpurun):
#   bash tools/knob_sweep.sh <tag> VAR v1 v2 ...    (env var VAR set to each value; "-" = unset)
set -uo pipefail
OUT=gpurun_out/${1:-knob}
VAR=$2
shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = "-" ]; then unset "$VAR"; else export "$VAR=$v"; fi
    timeout -k 10 120 python3 tools/c5run.py C5 C5wide H174 > "$OUT/$v.$rep.jsonl" 2> "$OUT/$v.$rep.err" || exit $?
    echo "$rep $VAR=$v $(python3 -c "import json; print([(d['name'], d['warm_s'], round(d['level_solo_ms'],1)) for d in map(json.loads, open('$OUT/$v.$rep.jsonl'))])")"
  done
done
unset "$VAR"
