"""Where the certified end-to-end leg's certification time goes
(s2lc_batch_results_flat on a warm C4 batch of 10k collector histories).

    python tools/cert_probe.py [histories]

One JSON line per measurement: verdicts only (no witnesses), the full
certification at several S2LC_THREADS, and the full certification into a
pre-touched witness buffer (no first-touch page faults in the timed call).
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    threads = min(16, os.cpu_count() or 1)
    ck = s2.Checker()
    b = None
    for first in (10 ** 6, 2 * 10 ** 6):
        hs = s2.load_many([s2.simulate_jsonl(**W.c4_params(sd)) for sd in range(first, first + n)], threads=threads)
        if b is None:
            b = ck.batch(hs)
        else:
            b.load(hs)
        b.run()
        b.results_flat(with_witness=True)
    cap = b.stats()["n_ops_total"]
    lib = s2.lib()

    def flat(ids, want):
        o = {k: np.zeros(n, t) for k, t in (("v", np.int32), ("r", np.int32), ("c", np.uint64), ("d", np.uint64))}
        offs = np.zeros(n + 1, np.uint64)
        p = lambda a: a.ctypes.data
        t0 = time.perf_counter()
        rc = lib.s2lc_batch_results_flat(ck._ctx, b._b, p(o["v"]), p(o["r"]), p(o["c"]), p(o["d"]),
                                         p(ids) if want else None, cap if want else 0, p(offs))
        t1 = time.perf_counter()
        assert rc == 0, rc
        return t1 - t0, int(offs[-1])

    def rep(tag, fn, k=7):
        ts = []
        for _ in range(k):
            ts.append(fn())
        ts.sort()
        print(json.dumps({"what": tag, "ms_min": round(ts[0] * 1e3, 3), "ms_med": round(ts[len(ts) // 2] * 1e3, 3),
                          "n_ops_total": cap}), flush=True)

    touched = np.ones(cap, np.int64)
    rep("verdicts_only", lambda: flat(touched, False)[0])
    for th in (1, 4, 8, 16, 24, 32):
        os.environ["S2LC_THREADS"] = str(th)
        rep(f"certify_pretouched_t{th}", lambda: flat(touched, True)[0])
    os.environ["S2LC_THREADS"] = "16"
    rep("certify_fresh_zeros_t16", lambda: flat(np.zeros(cap, np.int64), True)[0])
    import hashlib
    r = b.results_flat(with_witness=True)
    print(json.dumps({"what": "digest", "lib": os.path.basename(s2.LIB_PATH),
                      "sha": hashlib.sha256(b"".join(r[k].tobytes() for k in ("verdict", "witness_offs", "witness_ids"))).hexdigest()[:16],
                      "ok": int((r["verdict"] == s2.S2LC_OK).sum())}), flush=True)
    rep("results_flat_py_t16", lambda: (lambda t0: (b.results_flat(with_witness=True), time.perf_counter() - t0)[1])(
        time.perf_counter()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
