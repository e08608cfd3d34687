#!/bin/bash
# GPU tests of the 32-byte record paths, then C4 + end-to-end bench lines with
# and without them (S2LC_PACK_SMALL=0), alternated twice (from the repo root
# via gpurun):   bash tools/e2e_small_ab.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:-e2e_small}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_u64.py \
  tests/test_engines.py tests/test_c4_full.py > "$OUT/pytest.txt" 2>&1 || { tail -5 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-c5 --no-small --no-cpu-baseline > "$OUT/b$r.json" 2> "$OUT/b$r.err" || exit 1
  S2LC_PACK_SMALL=0 timeout -k 10 300 python3 bench.py --no-c5 --no-small --no-cpu-baseline > "$OUT/o$r.json" 2> "$OUT/o$r.err" || exit 1
done
