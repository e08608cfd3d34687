#!/bin/bash
# C4 parity (full batch, packed engines, GPU parity cases) + step overhead
set -uo pipefail
OUT=gpurun_out/${1:-itf}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_c4_full.py tests/test_gpu.py tests/test_cache.py \
  tests/test_engines.py -k "${2:-c4 or packed or reference or simulated or random or configs or flat or cache or timeout or witness}" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
S2LC_STEP_TIMING=1 timeout -k 10 120 python3 tools/step_overhead.py > "$OUT/step.json" 2> "$OUT/step.err" || exit $?
cat "$OUT/step.json"; tail -1 "$OUT/step.err"
