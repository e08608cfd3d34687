"""bench.py on the GPU: one short run, and the JSON line's contract (the
driver parses it): metric/value/unit, steps/warmup, roofline of the dominant
kernel, cpu_baseline with its core count, and every C4 verdict decided."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--histories", "2000",
           "--no-c5", "--no-e2e", "--no-small", "--cpu-seconds", "2"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["steps"] == 2 and d["warmup"] == 1 and d["n_gpus"] == 1 and d["unit"] == "histories/s"
    assert d["value"] > 0 and abs(d["value"] - 2000 * 2 / (d["ms_per_step"] * 2e-3)) / d["value"] < 0.01
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0
    assert cb["parity"]["verdict_mismatches"] == 0 and cb["parity"]["checked"] > 0
    assert d["verdicts"]["Unknown"] == 0 and d["verdicts"]["Ok"] + d["verdicts"]["Illegal"] == 2000
