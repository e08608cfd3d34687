#!/bin/bash
# Per-partitioned-round cost on one GPU (RCCL self-exchange, every round
# partitioned: wide = 0) against the single-GPU level search of the same
# history (from the repo root, via gpurun):  bash tools/dist_overhead.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:-dov}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/c5run.py H174 C5wide > "$OUT/single.jsonl" 2> "$OUT/single.err" || exit $?
for mode in "" "--sized"; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 tools/dist_c5.py --selfx --wide 0 $mode H174 C5wide >> "$OUT/wide0.jsonl" 2>> "$OUT/wide0.err" || exit $?
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
single = {d["name"]: d for d in map(json.loads, open(f"{out}/single.jsonl"))}
for l in open(f"{out}/wide0.jsonl"):
    if not l.startswith("{"):
        continue
    d = json.loads(l)
    s = single[d["name"]]
    over = (d["wall_s"] - s["warm_s"]) / max(1, d["rounds"]) * 1e6
    print(d["name"], "sized" if d["sized"] else "x", "rep", d["rep"], "wall", d["wall_s"], "single", s["warm_s"],
          "rounds", d["rounds"], "overhead_us_per_round", round(over, 1), "reruns", d["xreruns"])
PY
