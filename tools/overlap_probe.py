"""Do consecutive C4 batch runs overlap on one GPU? K steps of a 10k-history
batch run serially on one context, then the same K steps split over T host
threads, each with its own context (stream) and device batch, whose launches
the GPU runs concurrently (the ctypes call releases the GIL). One JSON line
per mode: histories/s over the wall time of all K steps.
    python tools/overlap_probe.py [steps] [threads ...]"""
import json
import os
import sys
import threading
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
modes = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
n = 10000
ctxs, batches = [], []
for t in range(max(modes)):
    c = s2.Checker()
    b = c.batch(W.c4_histories(n, first_seed=t * n))
    for _ in range(3):
        b.run()
    ctxs.append(c)
    batches.append(b)
for T in modes:
    steps = [K // T + (1 if i < K % T else 0) for i in range(T)]
    bar = threading.Barrier(T + 1)

    def work(i):
        bar.wait()
        for _ in range(steps[i]):
            batches[i].run()

    th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
    for x in th:
        x.start()
    bar.wait()
    t0 = time.perf_counter()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    ver = [sum(1 for r in batches[i].results(with_witness=False) if r.verdict == "Ok") for i in range(T)]
    print(json.dumps({"threads": T, "steps": K, "wall_s": round(wall, 4), "ms_per_step": round(1e3 * wall / K, 4),
                      "histories_per_s": round(n * K / wall, 1), "ok_per_batch": ver,
                      "kernel_ms_last": [round(batches[i].stats()["kernel_ms"], 4) for i in range(T)]}), flush=True)
