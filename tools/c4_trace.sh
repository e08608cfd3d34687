#!/bin/bash
# C4 step overhead and the kernel timeline of a few steps (rocprofv3 kernel trace)
set -euo pipefail
OUT=gpurun_out/${1:-c4trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
S2LC_STEP_TIMING=1 timeout -k 10 120 python3 tools/step_overhead.py > "$OUT/step.json" 2> "$OUT/step.err"
cat "$OUT/step.json"; tail -1 "$OUT/step.err"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o c4 -- \
  python3 bench.py --no-cpu-baseline --no-c5 --no-small --no-e2e --steps 5 --warmup 1 > "$OUT/bench.json" 2> "$OUT/trace.err"
python3 tools/trace_gaps.py "$OUT/trace"
