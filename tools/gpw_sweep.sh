#!/bin/bash
# lane groups per wave (S2LC_PACK_GPW; unset: the host's choice) vs the packed
# launch time over batch sizes (diagnostics)
set -uo pipefail
OUT=gpurun_out/${1:-gpw}
mkdir -p "$OUT"
for g in auto 1 2 4; do
  if [ "$g" = auto ]; then unset S2LC_PACK_GPW; else export S2LC_PACK_GPW=$g; fi
  timeout -k 10 200 python3 tools/pack_sweep.py 1 4 64 1000 2500 4000 6000 10000 > "$OUT/gpw_$g.jsonl" 2> "$OUT/gpw_$g.err" || exit $?
  echo "gpw=$g $(python3 -c "import json; print([(json.loads(l)['histories'], json.loads(l)['launch_ms']) for l in open('$OUT/gpw_$g.jsonl')])")"
done
