#!/bin/bash
# C4 launch times per environment setting (pack grid knobs), alternated twice
# (from the repo root via gpurun):
#   bash tools/pack_env_ab.sh <tag> "S2LC_PACK_BPC=1" "S2LC_PACK_BPC=2 S2LC_PACK_GPW=2" ...
# ("-" = no extra setting). Optional S2LC_LIB in the caller's environment.
set -uo pipefail
OUT=gpurun_out/${1:-packenv}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=()
    [ "$v" != "-" ] && read -r -a envs <<< "$v"
    env "${envs[@]}" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-c5 --no-small \
      --no-e2e --no-cpu-baseline > "$OUT/e$i.$rep.json" 2> "$OUT/e$i.$rep.err" || { echo "[$v] failed"; tail -3 "$OUT/e$i.$rep.err"; exit 1; }
    echo "$rep [$v] $(python3 -c "import json; d=json.load(open('$OUT/e$i.$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['verdicts'])")"
  done
done
