#!/bin/bash
# GPU-box profiling recipe (run through gpurun from the repo root):
#   bash profiles/collect.sh <tag>
# 1. bench.py (default run)                       -> gpurun_out/<tag>/bench.json
# 2. rocprofv3 --kernel-trace --stats, C4 only     -> gpurun_out/<tag>/stats/
# 3. two PMC passes (FETCH_SIZE, WRITE_SIZE)       -> gpurun_out/<tag>/pmc_*/
#    summarised for pack_kernel<16>                -> gpurun_out/<tag>/pmc_c4.json
# 4. rocprofv3 --kernel-trace --stats of C5        -> gpurun_out/<tag>/c5stats/
# Every GPU step has its own time limit; the first failure ends the script.
# (C5 under rocprofv3: the shipping cooperative launches, with tools/exit_hook.so (S2LC_EXIT_HOOK=1): the
# HIP runtime's own destructor faults at exit after cooperative launches under the profiler)
set -euo pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SHORT="--no-cpu-baseline --no-c5 --no-small --no-e2e --steps 3 --warmup 1"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o c4 -- \
  python3 bench.py $SHORT > "$OUT/stats_bench.json" 2> "$OUT/stats.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o c4 -- \
  python3 bench.py $SHORT > "$OUT/pmc_fetch_bench.json" 2> "$OUT/pmc_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o c4 -- \
  python3 bench.py $SHORT > "$OUT/pmc_write_bench.json" 2> "$OUT/pmc_write.err"
python3 profiles/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_c4.json" "pack_kernel<16>" "$OUT/pmc_fetch_bench.json"
S2LC_EXIT_HOOK=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5stats" -o c5 -- \
  python3 tools/c5run.py C5 > "$OUT/c5run.log" 2> "$OUT/c5stats.err"
