#!/bin/bash
# C5-class timings per library variant (S2LC_LIB), alternated twice (diagnostics):
#   bash tools/lib_ab.sh <tag> lib_a.so lib_b.so ...
set -uo pipefail
OUT=gpurun_out/${1:-ab}
shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    S2LC_LIB=$PWD/s2_verification_amd/$v timeout -k 10 120 python3 tools/c5run.py C5 C5wide H174 > "$OUT/$v.$rep.jsonl" 2> "$OUT/$v.$rep.err" || { echo "$v failed"; exit 1; }
    echo "$rep $v $(python3 -c "import json; print([(d['name'], d['verdict'], d['warm_s'], round(d['level_solo_ms'],1)) for d in map(json.loads, open('$OUT/$v.$rep.jsonl'))])")"
  done
done
