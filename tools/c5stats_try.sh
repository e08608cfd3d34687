#!/bin/bash
# C5 kernel stats under rocprofv3: plain persistent launches first, then
# cooperative ones (the r03a run faulted at exit, after the profiler's output)
set -euo pipefail
OUT=gpurun_out/${1:-c5try}
mkdir -p "$OUT"
export TMPDIR=/tmp
S2LC_PERSIST_PLAIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/plain" -o c5 -- \
  python3 tools/c5run.py C5 > "$OUT/plain.log" 2> "$OUT/plain.err"
echo plain ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/coop" -o c5 -- \
  python3 tools/c5run.py C5 > "$OUT/coop.log" 2> "$OUT/coop.err"
echo coop ok
