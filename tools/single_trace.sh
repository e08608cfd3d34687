#!/bin/bash
# Kernel trace of the single-GPU level search on named histories (persistent
# rounds as plain launches: S2LC_PERSIST_PLAIN=1), for the
# per-round costs of its host-enqueued rounds. From the repo root, via gpurun:
#   bash tools/single_trace.sh <tag> C5wide [C5 ...]
set -uo pipefail
OUT=gpurun_out/${1:-strace}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp S2LC_PERSIST_PLAIN=1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
  python3 tools/c5run.py "$@" > "$OUT/run.jsonl" 2> "$OUT/run.err"
rc=$?
cat "$OUT/run.jsonl"
find "$OUT/prof" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
exit $rc
