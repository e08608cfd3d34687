"""(round 6, measured with a temporary S2LC_TRACE_CAP knob, since removed: the pool size
made no difference) s2-porcupine -file=C1 per process (median of 9) with the default trace
pool (2^28 entries, 2 GiB) and a small one (S2LC_TRACE_CAP), with the CLI's
own phase split (S2LC_CLI_TIMING / S2LC_CREATE_TIMING)."""
import json
import os
import statistics
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
cli = os.path.join(ROOT, "s2_verification_amd", "s2-porcupine")
path = os.path.join(HERE, "c1.jsonl")
for rep in range(2):
    for cap in (None, "65536", "1048576"):
        env = dict(os.environ, S2LC_CLI_TIMING="1", S2LC_CREATE_TIMING="1")
        if cap:
            env["S2LC_TRACE_CAP"] = cap
        ts, ph = [], []
        for _ in range(9):
            t0 = time.perf_counter()
            p = subprocess.run([cli, "-file=" + path], capture_output=True, text=True, timeout=60, env=env)
            ts.append(1e3 * (time.perf_counter() - t0))
            for ln in p.stderr.splitlines():
                if ln.startswith('{"cli_timing_ms"'):
                    ph.append(json.loads(ln)["cli_timing_ms"])
        main = statistics.median([x["main"] for x in ph]) if ph else None
        print(json.dumps({"trace_cap": cap or "default", "process_ms": round(statistics.median(ts), 1),
                          "min_ms": round(min(ts), 1), "main_ms": main,
                          "outside_main_ms": round(statistics.median(ts) - main, 1) if main else None,
                          "phases_last": ph[-1] if ph else None, "rc": p.returncode}), flush=True)
