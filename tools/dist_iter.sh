#!/bin/bash
# Distributed-search iteration on the GPU box (from the repo root, via gpurun):
#   bash tools/dist_iter.sh <tag>
# the distributed GPU tests, then per-partitioned-round cost on one GPU (RCCL
# self-exchange) host-free vs the round-3 sized exchange, at two widths.
set -uo pipefail
TAG=${1:-dist}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist.py -m gpu \
  > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
for w in 4096 1024; do
  for mode in "" "--sized"; do
    timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29531 tools/dist_c5.py --selfx --wide $w $mode C5wide C5 >> "$OUT/selfx.jsonl" 2>> "$OUT/selfx.err" || exit $?
  done
done
cat "$OUT/selfx.jsonl"
