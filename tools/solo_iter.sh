#!/bin/bash
# Solo-round iteration (from the repo root via gpurun): level parity on the
# current build, C5-class A/B against a baseline library, a PROF pass.
#   bash tools/solo_iter.sh <tag> [baseline.so]
set -uo pipefail
TAG=${1:-solo}
BASE=${2:-libs2lincheck_base.so}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_level.py tests/test_engines.py \
  -k "hard or level or solo or persist or staging or rerun" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
bash tools/lib_ab.sh "$TAG/ab" "$BASE" libs2lincheck.so || exit $?
S2LC_LIB=$PWD/s2_verification_amd/libs2lincheck_prof.so timeout -k 10 120 python3 tools/c5run.py C5 H174 > "$OUT/prof.jsonl" 2> "$OUT/prof.txt" || exit $?
grep "solo" "$OUT/prof.txt" | head -8
