#!/bin/bash
# level-search parity (hard-history round counts in every round mode, level
# tests) + C5 timings (from the repo root via gpurun)
set -uo pipefail
OUT=gpurun_out/${1:-itc5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_level.py tests/test_engines.py \
  -k "${2:-hard or level or solo or persist or staging or rerun}" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/c5run.py C5 H174 C5bad C5wide > "$OUT/c5run.jsonl" 2> "$OUT/c5run.err" || exit $?
python3 -c "
import json
for l in open('$OUT/c5run.jsonl'): d=json.loads(l); print(d['name'], d['verdict'], d['warm_s'], d['level_rounds'])"
