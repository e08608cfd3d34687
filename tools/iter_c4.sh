#!/bin/bash
# One C4 iteration on the GPU box (from the repo root, via gpurun):
#   bash tools/iter_c4.sh <tag> [pytest -k expression]
# parity of the packed kernels (full C4 batch + packed round counts + GPU
# parity cases), then the launch-time sweep; stops at the first failure.
set -uo pipefail
TAG=${1:-iter}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_c4_full.py tests/test_gpu.py tests/test_engines.py ${K:+-k "$K"} > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 240 python3 tools/pack_sweep.py 1 4 64 1000 10000 > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
rc2=$?
cat "$OUT/sweep.jsonl"
[ $rc -eq 0 ] && exit $rc2 || exit $rc
