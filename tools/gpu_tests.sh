#!/bin/bash
# The whole -m gpu suite on the GPU box (from the repo root, via gpurun):
#   bash tools/gpu_tests.sh <tag> [extra pytest args]
set -uo pipefail
TAG=${1:-gt}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1080 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -5 "$OUT/pytest.txt"
exit $rc
