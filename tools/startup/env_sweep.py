"""HIP runtime start-up cost per environment setting (the s2-porcupine CLI
is one process per history, main.go:568-640): tools/startup/hip_startup in
mode 1 (hipGetDeviceCount, _exit) and mode 4 (stream + 2 GiB + one kernel),
median of 7 processes per setting; then the CLI itself on C1 per setting.
    python tools/startup/env_sweep.py [cli_jsonl]"""
import json
import os
import statistics
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
exe = os.path.join(HERE, "hip_startup")
SETTINGS = [{}, {"HSA_ENABLE_SDMA": "0"}, {"ROCR_VISIBLE_DEVICES": "0"}, {"HIP_VISIBLE_DEVICES": "0"},
            {"HSA_ENABLE_INTERRUPT": "0"}, {"HIP_ENABLE_DEFERRED_LOADING": "1"},
            {"HIP_ENABLE_DEFERRED_LOADING": "0"}, {"AMD_DIRECT_DISPATCH": "0"},
            {"HSA_ENABLE_SDMA": "0", "ROCR_VISIBLE_DEVICES": "0"}]


def timed(cmd, env, reps=7):
    ts, last = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=60, env=env)
        ts.append(1e3 * (time.perf_counter() - t0))
        if p.returncode not in (0, 1):
            return None, p.returncode, p.stderr[-300:]
        last = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else ""
    return round(statistics.median(ts), 1), 0, last


cli = os.path.join(ROOT, "s2_verification_amd", "s2-porcupine")
jsonl = sys.argv[1] if len(sys.argv) > 1 else None
for st in SETTINGS:
    env = dict(os.environ, **st)
    row = {"env": st}
    for mode in (1, 4):
        ms, rc, last = timed([exe, str(mode), "1"], env)
        row[f"mode{mode}_ms"] = ms if ms is not None else f"rc {rc}: {last}"
    if jsonl:
        ms, rc, last = timed([cli, "-file=" + jsonl], env, reps=5)
        row["cli_c1_ms"] = ms if ms is not None else f"rc {rc}: {last}"
    print(json.dumps(row), flush=True)
