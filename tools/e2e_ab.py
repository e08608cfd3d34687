"""bench.py's certified end-to-end leg alone (collector JSONL in memory ->
verdicts + certified witnesses, cold / warm / cache passes), one JSON line.
For A/B runs of the host pipeline on one box, e.g. the history pool:

    python tools/e2e_ab.py [histories]                 (default 10000)
    S2LC_HISTORY_POOL_MB=0 python tools/e2e_ab.py
"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import s2_verification_amd as s2
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    args = types.SimpleNamespace(histories=n)
    out = bench.end_to_end_leg(args, s2.Checker(), 0, 1)
    out["pool_mb"] = os.environ.get("S2LC_HISTORY_POOL_MB", "default")
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
