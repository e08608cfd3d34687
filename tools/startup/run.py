"""Time tools/startup/hip_startup per mode as whole processes (median of 5)."""
import json
import os
import statistics
import subprocess
import sys
import time

exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip_startup")
for mode in range(5):
    for fast in (0, 1):
        ts, inner = [], None
        for _ in range(5):
            t0 = time.perf_counter()
            p = subprocess.run([exe, str(mode), str(fast)], capture_output=True, text=True, timeout=60)
            ts.append(1e3 * (time.perf_counter() - t0))
            if p.returncode:
                print(json.dumps({"mode": mode, "rc": p.returncode, "err": p.stderr[-300:]}))
                sys.exit(1)
            inner = json.loads(p.stdout)
        print(json.dumps({"mode": mode, "fast_exit": fast, "process_ms": round(statistics.median(ts), 1), "last": inner}),
              flush=True)
