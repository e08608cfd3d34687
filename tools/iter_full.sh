#!/bin/bash
# parity subset + groups-per-wave sweep + bench (from the repo root, via gpurun)
set -uo pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/iter_c4.sh "$TAG/iter" "${2:-c4 or packed or reference or simulated or random or configs or flat}" || exit $?
bash tools/gpw_sweep.sh "$TAG/gpw" || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['kernel_ms'], 'c5', d['c5'].get('seconds'), 'e2e', d.get('end_to_end',{}).get('histories_per_sec'), 'cache', d.get('end_to_end',{}).get('from_cache_histories_per_sec'))"
