#!/bin/bash
# Kernel stats + the HBM-traffic PMC passes the bench's roofline lines read
# (run through gpurun from the repo root after any kernel-source change):
#   bash profiles/collect_traffic.sh <tag>
# C4 (bench.py, C4 leg only): kernel stats, FETCH_SIZE, WRITE_SIZE
#   -> python3 profiles/pmc_summary.py ... > profiles/<round>/pmc_c4.json
# C5 (tools/c5run.py C5, cold + warm): kernel stats (cooperative launches, with
# the profiling exit hook), FETCH_SIZE, WRITE_SIZE, EA atomics
#   -> python3 profiles/pmc_c5.py gpurun_out/<tag> > profiles/<round>/pmc_c5.json
# One counter group per rocprofv3 run; every GPU step has its own time limit
# and the first failure ends the script.
set -euo pipefail
TAG=${1:-traffic}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SHORT="--no-cpu-baseline --no-c5 --no-small --no-e2e --steps 3 --warmup 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o c4 -- \
  python3 bench.py $SHORT > "$OUT/stats_bench.json" 2> "$OUT/stats.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o c4 -- \
  python3 bench.py $SHORT > "$OUT/pmc_fetch_bench.json" 2> "$OUT/pmc_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o c4 -- \
  python3 bench.py $SHORT > "$OUT/pmc_write_bench.json" 2> "$OUT/pmc_write.err"
S2LC_EXIT_HOOK=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5stats" -o c5 -- \
  python3 tools/c5run.py C5 > "$OUT/c5run.log" 2> "$OUT/c5stats.err"
for grp in "c5_fetch FETCH_SIZE TCC_ATOMIC" "c5_write WRITE_SIZE TCC_ATOMIC" "c5_atomic TCC_ATOMIC TCC_EA0_ATOMIC"; do
  set -- $grp
  name=$1; shift
  S2LC_EXIT_HOOK=1 timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    python3 tools/c5run.py C5 > "$OUT/$name.out" 2> "$OUT/$name.err"
done
echo done > "$OUT/DONE"
