#!/bin/bash
# C5 kernel stats (rocprofv3 --kernel-trace --stats over tools/c5run.py C5,
# two searches) then the PMC passes of profiles/collect_pmc.sh
set -euo pipefail
TAG=${1:-c5prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5stats" -o c5 -- \
  python3 tools/c5run.py C5 > "$OUT/c5run.log" 2> "$OUT/c5stats.err"
bash profiles/collect_pmc.sh "$TAG/pmc"
python3 profiles/pmc_c5.py "$OUT/pmc" > "$OUT/pmc_c5.json"
python3 profiles/pmc_sq.py "$OUT/pmc" > "$OUT/pmc_sq.json"
