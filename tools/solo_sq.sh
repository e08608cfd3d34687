#!/bin/bash
# SQ counters of the solo rounds alone: lv_persist with ONE workgroup
# (S2LC_PERSIST_GRID=1; frontiers wider than 4 go host-driven), H174 (from the
# repo root via gpurun):  bash tools/solo_sq.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:-solosq}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  S2LC_PERSIST_GRID=1 S2LC_PERSIST_PLAIN=1 timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    python3 tools/c5run.py H174 > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "$name failed"; tail -3 "$OUT/$name.err"; return 1; }
}
run sq_a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU || exit 1
run sq_b SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS || exit 1
run sq_c SQ_IFETCH SQ_INSTS_SENDMSG SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT || true
python3 profiles/pmc_sq.py "$OUT" > "$OUT/summary.json"
python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k,v in d.items():
    if 'persist' in k or k.startswith('sq'): print(k, json.dumps(v)[:1500])
"
