"""Where a C4 bench step's time goes besides the search kernel: wall time of
Batch.run() and Batch.stats() over many steps against the kernel's HIP-event
time (diagnostics; prints one JSON line)."""
import json
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402

hs = W.c4_histories(10000)
b = s2.Checker().batch(hs)
for _ in range(3):
    b.run()
n = 50
t_run = t_stats = k = 0.0
for _ in range(n):
    t0 = time.perf_counter()
    b.run()
    t1 = time.perf_counter()
    st = b.stats()
    t2 = time.perf_counter()
    t_run += t1 - t0
    t_stats += t2 - t1
    k += st["kernel_ms"]
print(json.dumps({"run_ms": round(1e3 * t_run / n, 4), "stats_ms": round(1e3 * t_stats / n, 4),
                  "kernel_ms": round(k / n, 4), "overhead_ms": round(1e3 * t_run / n - k / n, 4)}))
