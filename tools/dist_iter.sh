#!/bin/bash
# Distributed-search iteration on the GPU box (from the repo root, via gpurun):
#   bash tools/dist_iter.sh <tag> [widths...]
# the distributed GPU tests, the one-GPU rehearsal (self-exchange from `wide`)
# at each width, and the per-partitioned-round overhead (every round
# partitioned) against the single-GPU search.
set -uo pipefail
TAG=${1:-dist}
shift || true
WIDTHS=${*:-4096}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist.py -m gpu \
  > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
for w in $WIDTHS; do
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 tools/dist_c5.py --selfx --reps 3 --wide $w C5wide C5 >> "$OUT/selfx.jsonl" 2>> "$OUT/selfx.err" || exit $?
done
grep '^{' "$OUT/selfx.jsonl"
bash tools/dist_overhead.sh "$TAG/ov" > "$OUT/overhead.txt" 2>&1 || exit $?
cat "$OUT/overhead.txt"
