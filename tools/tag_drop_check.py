import os, sys, time
sys.path[:0] = ['.']
import s2_verification_amd as s2
from s2_verification_amd import workloads as W
h = W.config_history("H174")
for drop in ("0", "0xFFFFFF00", "0xFFFFFFF0", "0xFFFFFFFF"):
    os.environ["S2LC_TAG_DROP"] = drop
    os.environ["S2LC_NO_SOLO"] = "1"
    b = s2.Checker(round_counts=True).batch([h])
    b.check()
    t = time.time(); r = b.check()[0]; dt = time.time() - t
    print(drop, r.verdict, round(dt, 4), b.stats()["level_configs"], flush=True)
