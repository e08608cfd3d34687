#!/bin/bash
# Packed-kernel iteration on the GPU box (from the repo root, via gpurun):
#   bash tools/pack_iter.sh <tag> [baseline.so]
# parity of the packed kernels (full C4 batch, packed round counts, GPU parity
# cases), then the C4 launch sweep alternated twice between the baseline
# library and the current one, then the slowest histories alone.
set -uo pipefail
TAG=${1:-pk}
BASE=${2:-libs2lincheck_base.so}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_c4_full.py tests/test_gpu.py tests/test_engines.py -k "not hard and not level and not persist" \
  > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
bash tools/variant_sweep.sh "$TAG/vs1" "$BASE" libs2lincheck.so || exit $?
bash tools/variant_sweep.sh "$TAG/vs2" "$BASE" libs2lincheck.so || exit $?
timeout -k 10 200 python3 tools/pack_single.py 120 > "$OUT/single.jsonl" 2> "$OUT/single.err" || exit $?
head -5 "$OUT/single.jsonl"
S2LC_LIB=$PWD/s2_verification_amd/$BASE timeout -k 10 200 python3 tools/pack_single.py 120 > "$OUT/single_base.jsonl" 2> "$OUT/single_base.err" || exit $?
head -5 "$OUT/single_base.jsonl"
