"""Verdicts of the hard single histories (workloads.CONFIGS C5, C5bad, H174,
H212, C5wide) from the CPU reduced search (oracle/reduced.c), committed as
tests/golden/hard_reduced.json so the GPU tests need not re-run minutes of CPU
search. Also records a fingerprint of each history's event list, so a changed
simulator is caught instead of silently comparing against stale verdicts.

Run here (not on the GPU box): python tests/golden/make_hard_golden.py
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


def main(names):
    path = os.path.join(HERE, "hard_reduced.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        h = W.config_history(name)
        t = time.time()
        v, st = orc.check_reduced(orc.from_s2lc_numpy(h.events_numpy()))
        out[name] = {"verdict": v, "digest": config_digest(name), "info": h.info(),
                     "reduced": {k: st[k] for k in ("configs", "rounds", "max_frontier", "children")},
                     "cpu_seconds": round(time.time() - t, 1)}
        print(name, out[name], flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["H174", "H212", "C5bad", "C5", "C5wide"])
