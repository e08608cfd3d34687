"""JSONL decode throughput on the host (no GPU): s2lc_load_jsonl_many over the
C4 histories at several thread counts, three passes each, the previous pass's
histories released first (the bench's steady state).
    python tools/decode_box.py [n_histories]"""
import json
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
blobs = [s2.simulate_jsonl(**W.c4_params(sd)) for sd in range(2 * 10 ** 6, 2 * 10 ** 6 + n)]
nb = sum(len(b) for b in blobs)
for th in (1, 4, 16):
    sub = blobs if th > 1 else blobs[: max(1, n // 10)]
    sb = sum(len(b) for b in sub)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        hs = s2.load_many(sub, threads=th)
        ts.append(time.perf_counter() - t)
        del hs
    k = min(ts)
    print(json.dumps({"threads": th, "histories": len(sub), "seconds": round(k, 4), "GB_per_s": round(sb / k * 1e-9, 2),
                      "us_per_history_thread": round(k * th / len(sub) * 1e6, 1), "all": [round(x, 4) for x in ts]}), flush=True)
