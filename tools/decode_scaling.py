"""Collector-JSONL decode throughput (s2lc_load_jsonl_many) on the host cores:
threads x passes, histories of C4's shape. The second and later passes decode
into the storage the previous pass released (the history pool,
S2LC_HISTORY_POOL_MB; run with S2LC_HISTORY_POOL_MB=0 for the C heap).

    python tools/decode_scaling.py [n] [threads ...]      (default 10000 1 16)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    threads = [int(x) for x in sys.argv[2:]] or [1, 16]
    blobs = [s2.simulate_jsonl(**W.c4_params(sd)) for sd in range(2 * 10 ** 6, 2 * 10 ** 6 + n)]
    nb = sum(len(b) for b in blobs)
    for th in threads:
        m = n if th > 1 else max(1, n // 10)
        sub = blobs[:m]
        sb = sum(len(b) for b in sub)
        passes = []
        for _ in range(4):
            t0 = time.perf_counter()
            hs = s2.load_many(sub, threads=th)
            dt = time.perf_counter() - t0
            passes.append(round(dt, 4))
            del hs
        best = min(passes[1:])
        print(json.dumps({"threads": th, "histories": m, "jsonl_bytes": sb, "pool_mb": os.environ.get("S2LC_HISTORY_POOL_MB", "default"),
                          "pass_s": passes, "GBps_warm": round(sb / best / 1e9, 2), "histories_per_s_warm": round(m / best)}),
              flush=True)
    return 0 if nb else 1


if __name__ == "__main__":
    sys.exit(main())
