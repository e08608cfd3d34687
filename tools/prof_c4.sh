#!/bin/bash
# C4 packed-kernel anatomy on the GPU box (run from the repo root via gpurun):
#   bash tools/prof_c4.sh <tag>
# 1. tools/pack_sweep.py: launch time vs the longest history's round chain
# 2. the same with the PROF library (per-phase cycles per round)
# 3. SQ counters of pack_kernel<16> at 1,000 and 10,000 histories
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-c4prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/pack_sweep.py > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
S2LC_LIB=$PWD/s2_verification_amd/libs2lincheck_prof.so timeout -k 10 240 python3 tools/pack_sweep.py 1 256 1000 10000 \
  > "$OUT/sweep_prof.jsonl" 2> "$OUT/sweep_prof.err"
for m in 1000 10000; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM \
    --output-format csv -d "$OUT/sq_a_$m" -o run -- python3 tools/pack_sweep.py $m > "$OUT/sq_a_$m.out" 2> "$OUT/sq_a_$m.err"
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES \
    --output-format csv -d "$OUT/sq_b_$m" -o run -- python3 tools/pack_sweep.py $m > "$OUT/sq_b_$m.out" 2> "$OUT/sq_b_$m.err"
done
