"""Decode of freshly generated collector JSONL against a second decode of the
same bytes (16 threads, 10k C4 histories): does the first read of new input
cost the decode more than the parse itself?

    python tools/decode_fresh.py [n]
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
    th = 16
    for rep in range(3):
        base = (3 + rep) * 10 ** 6
        blobs = [s2.simulate_jsonl(**W.c4_params(sd)) for sd in range(base, base + n)]
        ts = []
        for k in range(3):
            t0 = time.perf_counter()
            hs = s2.load_many(blobs, threads=th)
            ts.append(round(time.perf_counter() - t0, 4))
            del hs
        print(json.dumps({"rep": rep, "fresh_then_again_s": ts}), flush=True)
        del blobs
    return 0


if __name__ == "__main__":
    sys.exit(main())
