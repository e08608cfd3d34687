"""The whole C4 batch (BASELINE.json configs[3]: seeds 0..9999, the exact batch
bench.py times) checked on the CPU, committed as tests/golden/c4_verdicts.json:

  * per seed, porcupine's WGL restated (oracle/oracle.c or_check_wgl,
    computePartial on, like CheckEventsVerbose): verdict + cache inserts
    (porcupine's "configs explored");
  * per seed, the CPU reduced search (oracle/reduced.c, the GPU's rounds
    restated): verdict, rounds, unique configurations and a digest of the
    per-round unique-configuration counts;
  * a digest of the simulator's output for the whole batch (the events of
    every history), so a changed simulator is caught instead of compared
    against stale verdicts.

tests/test_c4_full.py runs the same 10,000 histories on the GPU and compares
every one of these. Run here (not on the GPU box):

    python tests/golden/make_c4_golden.py [n]
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

V = {"Ok": "O", "Illegal": "I", "Unknown": "U"}


def counts_digest(counts):
    """16 hex digits of sha256 over the per-round counts (u32 little endian)."""
    import numpy as np
    return hashlib.sha256(np.asarray(counts, dtype="<u4").tobytes()).hexdigest()[:16]


def _work(seeds):
    import oracle as orc
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    out = []
    for sd in seeds:
        h = s2.simulate_history(**W.c4_params(sd))
        ea = orc.from_s2lc_numpy(h.events_numpy(), owner=h)
        w, wst = orc.check_wgl(ea, compute_partial=True)
        r, rst = orc.check_reduced(ea, round_counts=True)
        out.append([sd, V[w], wst["cache_inserts"], V[r], rst["rounds"], rst["configs"],
                    counts_digest(rst["round_counts"])])
    return out


def batch_digest(n):
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    hsh = hashlib.sha256()
    for sd in range(n):
        hsh.update(s2.simulate_jsonl(**W.c4_params(sd)))
    return hsh.hexdigest()[:32]


def main(n=10000):
    t = time.time()
    chunks = [list(range(i, min(n, i + 250))) for i in range(0, n, 250)]
    with mp.get_context("spawn").Pool(min(8, os.cpu_count() or 1)) as pool:
        rows = [r for part in pool.map(_work, chunks) for r in part]
    rows.sort()
    out = {"n": n, "first_seed": 0,
           "simulator_jsonl_sha256": batch_digest(n),
           "columns": ["seed", "wgl_verdict", "wgl_cache_inserts", "reduced_verdict", "reduced_rounds",
                       "reduced_configs", "round_counts_sha256_16"],
           "rows": [r[1:] for r in rows],
           "cpu_seconds": round(time.time() - t, 1)}
    assert all(r[1] == r[3] for r in rows), "WGL and the reduced search disagree"
    with open(os.path.join(HERE, "c4_verdicts.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print({k: out[k] for k in ("n", "simulator_jsonl_sha256", "cpu_seconds")},
          {v: sum(1 for r in rows if r[1] == v) for v in "OIU"})


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10000)
