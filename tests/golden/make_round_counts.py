"""Per-round unique-configuration counts of the CPU reduced search
(oracle/reduced.c) on the hard single histories, under reduction ablations,
committed as tests/golden/hard_round_counts.json. The GPU engines must produce
the same verdict AND the same count in every completed round (tests/
test_engines.py): same reductions => same configuration set per round, so
this pins the search itself, not only its final bit.

Which ablations: only those whose search stays small on these histories.
Switching P1, P4 (on the Ok histories) or the indefinite deferral off makes
them explode (tens of millions of configurations); those switches are
exercised on the mid-size histories instead, live in the test.

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

CASES = {"H174": [0, 2], "H212": [0, 2], "C5bad": [0, 2, 4], "C5wide": [0]}


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
    with open(path, "w") as f:
        json.dump(out, f, sort_keys=True, separators=(",", ":"))


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
