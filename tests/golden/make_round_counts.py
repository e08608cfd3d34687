"""Per-round unique-configuration counts of the CPU reduced search
(oracle/reduced.c) on the hard single histories, under reduction ablations,
committed as tests/golden/hard_round_counts.json. The GPU engines must produce
the same verdict AND the same count in every completed round (tests/
test_engines.py): same reductions => same configuration set per round, so
this pins the search itself, not only its final bit.

Which ablations: complete searches for those that stay small on these
histories (all on, P2 off, P4 off on C5bad). Switching P1 or the indefinite
deferral off makes them explode: with P1 off, H174 passes 66 M unique
configurations by round 1,037 of ~10,300 (frontier 7.4 M) and C5bad 61 M by
round 668; with the deferral off neither passes round ~1,000 within 30 CPU
minutes. For those (PREFIX) the search runs under a configuration budget
(or_check_reduced's max_configs) and the fixture keeps the counts of every
round completed before it ran out ("complete": false): the GPU, under a
smaller budget, must reproduce that prefix round by round. The whole-search
P1 / deferral ablations run on A144 / A160 (> 128 chains, level search: P1 off
4.9 M configurations, deferral off 36 k / 4.2 M) and on the mid-size
histories, live in the test.

Run here (not on the GPU box): python tests/golden/make_round_counts.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as orc  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402
from helpers import config_digest  # noqa: E402

CASES = {"H174": [0, 2], "H212": [0, 2], "C5bad": [0, 2, 4], "C5wide": [0],
         # > 128 chains, whole-search P1 / deferral ablations (A160: P1 or P4 off explodes)
         "A144": [0, 1, 2, 4, 8], "A160": [0, 2, 8]}
# (reductions_off, configuration budget): prefix fixtures of exploding ablations
PREFIX = {"H174": [(1, 60_000_000), (8, 30_000_000)], "C5bad": [(1, 60_000_000), (8, 30_000_000)]}


def main(names):
    path = os.path.join(HERE, "hard_round_counts.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        offs = CASES[name]
        h = W.config_history(name)
        ea = orc.from_s2lc_numpy(h.events_numpy(), owner=h)
        out[name] = {"digest": config_digest(name)}
        for off in offs:
            t = time.time()
            v, st = orc.check_reduced(ea, reductions_off=off, round_counts=True)
            out[name][str(off)] = {"verdict": v, "rounds": st["rounds"], "configs": st["configs"],
                                   "counts": st["round_counts"], "cpu_seconds": round(time.time() - t, 1)}
            print(name, off, v, st["rounds"], st["configs"], flush=True)
        for off, budget in PREFIX.get(name, []):
            t = time.time()
            v, st = orc.check_reduced(ea, reductions_off=off, round_counts=True, max_configs=budget)
            out[name][f"{off}p"] = {"verdict": v, "budget": budget, "complete": v != "Unknown",
                                     "rounds": st["rounds"], "configs": st["configs"], "max_frontier": st["max_frontier"],
                                     "counts": st["round_counts"], "cpu_seconds": round(time.time() - t, 1)}
            print(name, f"{off}p", v, st["rounds"], st["configs"], flush=True)
    with open(path, "w") as f:
        json.dump(out, f, sort_keys=True, separators=(",", ":"))


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
