"""Where the C4 launch time goes: the longest history's chain of rounds (the
latency floor) versus issue throughput. For m in a sweep, the m C4 histories
with the most rounds (tests/golden/c4_verdicts.json, the CPU reduced search's
round counts) run as one batch; each line reports the packed launch's HIP-event
time, the batch's largest round count and the time per round of that longest
chain. m = 1 is one lone 16-lane group (no issue contention, no lockstep with
other groups of its wave).

    python tools/pack_sweep.py [m ...]      (default 1 4 64 256 1000 2500 5000 10000)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402

ref = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_verdicts.json")))
rounds = [r[3] for r in ref["rows"]]
order = sorted(range(len(rounds)), key=lambda i: -rounds[i])
ms = [int(x) for x in sys.argv[1:]] or [1, 4, 64, 256, 1000, 2500, 5000, 10000]
hs_all = {}
ck = s2.Checker()
for m in ms:
    seeds = order[:m]
    hs = [hs_all.setdefault(sd, s2.simulate_history(**W.c4_params(sd))) for sd in seeds]
    b = ck.batch(hs)
    for _ in range(2):
        b.run()
    t = []
    for _ in range(5):
        b.run()
        st = b.stats()
        t.append(st["pack16_ms"] + st["pack8_ms"])
    k = min(t)
    rmax = max(rounds[sd] for sd in seeds)
    print(json.dumps({"histories": m, "launch_ms": round(k, 4), "max_rounds": rmax,
                      "us_per_round_longest": round(1e3 * k / rmax, 3),
                      "mean_rounds": round(sum(rounds[sd] for sd in seeds) / m, 1),
                      "pack16": st["pack16_histories"], "pack8": st["pack8_histories"]}), flush=True)
