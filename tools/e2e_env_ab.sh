#!/bin/bash
# End-to-end (C4 JSONL -> certified verdicts) bench lines per environment
# setting, alternated twice (from the repo root via gpurun):
#   bash tools/e2e_env_ab.sh <tag> "-" "S2LC_CERT_PAIRS=0" ...     ("-" = no extra setting)
set -uo pipefail
OUT=gpurun_out/${1:-e2eenv}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=()
    [ "$v" != "-" ] && read -r -a envs <<< "$v"
    env "${envs[@]}" timeout -k 10 300 python3 bench.py --no-c5 --no-small --no-cpu-baseline --steps 5 --warmup 2 \
      > "$OUT/e$i.$rep.json" 2> "$OUT/e$i.$rep.err" || { echo "[$v] failed"; tail -3 "$OUT/e$i.$rep.err"; exit 1; }
    echo "$rep [$v] $(python3 -c "
import json; d=json.load(open('$OUT/e$i.$rep.json')); e=d['end_to_end']; w=e['warm']
print(e['histories_per_sec'], w['decode_s'], w['upload_s'], w['witness_replay_s'], e['cache']['histories_per_sec'], w['ok_without_witness'])")"
  done
done
