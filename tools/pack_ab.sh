#!/bin/bash
# C4 launch times per library variant (S2LC_LIB), alternated twice (from the
# repo root via gpurun):  bash tools/pack_ab.sh <tag> lib_a.so lib_b.so ...
set -uo pipefail
OUT=gpurun_out/${1:-packab}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    S2LC_LIB=$PWD/s2_verification_amd/$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-c5 --no-small \
      --no-e2e --no-cpu-baseline > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { echo "$v failed"; tail -3 "$OUT/$v.$rep.err"; exit 1; }
    echo "$rep $v $(python3 -c "import json; d=json.load(open('$OUT/$v.$rep.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['launch_ms'], d['verdicts'])")"
  done
done
