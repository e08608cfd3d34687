#!/bin/bash
# lane groups per wave (S2LC_PACK_GPW) x LPT-head histories run one per wave
# (S2LC_PACK_SOLO_N) vs the packed launch time (diagnostics)
set -uo pipefail
OUT=gpurun_out/${1:-gpw}
mkdir -p "$OUT"
for g in 2 4; do
  for s in 0 256 512 1024 2048; do
    S2LC_PACK_GPW=$g S2LC_PACK_SOLO_N=$s timeout -k 10 200 python3 tools/pack_sweep.py 1000 10000 > "$OUT/g${g}s${s}.jsonl" 2> "$OUT/g${g}s${s}.err" || exit $?
    echo "gpw=$g solo=$s $(python3 -c "import json,sys; print([json.loads(l)['launch_ms'] for l in open('$OUT/g${g}s${s}.jsonl')])")"
  done
done
