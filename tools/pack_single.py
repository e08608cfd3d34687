"""Which C4 histories bound the packed launch: each of the m C4 histories with
the most rounds (tests/golden/c4_verdicts.json) runs ALONE (a one-history
batch, one lone 16-lane group), and the lines report its launch time, rounds,
children, configurations and chain count, slowest first. The 10k launch can
finish no sooner than its slowest history alone.

    python tools/pack_single.py [m]      (default 200)
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
m = int(sys.argv[1]) if len(sys.argv) > 1 else 200
order = sorted(range(len(rounds)), key=lambda i: -rounds[i])[:m]
ck = s2.Checker()
rows = []
for sd in order:
    h = s2.simulate_history(**W.c4_params(sd))
    b = ck.batch([h])
    b.run()
    t = []
    for _ in range(4):
        b.run()
        st = b.stats()
        t.append(st["pack16_ms"] + st["pack8_ms"])
    r = b.results(with_witness=False)[0]
    info = h.info()
    rows.append({"seed": sd, "ms": round(min(t), 4), "rounds": r.rounds, "children": st["children_generated"],
                 "configs": r.configs_explored, "K": info["n_chains"], "n_ops": info["n_ops"],
                 "us_per_round": round(1e3 * min(t) / max(1, r.rounds), 3)})
rows.sort(key=lambda d: -d["ms"])
for d in rows:
    print(json.dumps(d), flush=True)
