#!/bin/bash
# Kernel trace of the distributed search's one-GPU rehearsal (one rank, RCCL
# self-exchange, partitioned rounds from `wide`), persistent rounds as plain
# launches (S2LC_PERSIST_PLAIN=1: no cooperative launch, whose HIP-runtime
# teardown faults under the profiler). From the repo root, via gpurun:
#   bash tools/dist_prof.sh <tag> [dist_c5.py args...]
set -uo pipefail
OUT=gpurun_out/${1:-dprof}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 S2LC_PERSIST_PLAIN=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 tools/dist_c5.py --reps 2 "$@" > "$OUT/run.jsonl" 2> "$OUT/run.err"
rc=$?
cat "$OUT/run.jsonl"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
head -20 "$OUT/kernel_stats.csv" 2>/dev/null
exit $rc
