"""The committed round-1 bench line keeps the bench.py contract, and its
roofline agrees with the rocprofv3 summary committed beside it.

CPU only: reads files under profiles/ (no GPU, no oracle)."""
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles", "r01f")


def _line(name):
    with open(os.path.join(PROF, name)) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_bench_line_fields():
    line = _line("bench_c4.json")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["config"]["workload"] == "C4"
    assert line["n_gpus"] == 1 and line["higher_is_better"] is True
    # value = histories per step / step time
    hist = line["config"]["histories_per_gpu"]
    assert abs(line["value"] - hist / (line["ms_per_step"] / 1e3)) / line["value"] < 0.01
    assert line["parity_sample"]["verdict_mismatches"] == 0
    cb = line["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0


def test_roofline_consistent():
    rl = _line("bench_c4.json")["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-4
    # achieved = algorithmic bytes per launch / launch time
    assert abs(rl["achieved"] - rl["algo_bytes_per_launch"] / (rl["launch_ms"] * 1e6)) / rl["achieved"] < 0.01
    # PMC traffic within a few percent of the algorithmic bytes (no wasted re-reads)
    assert rl["traffic_bytes_per_launch"] < 1.1 * rl["algo_bytes_per_launch"]


def test_rocprof_agrees_with_hip_events():
    rl = _line("bench_c4.json")["roofline"]
    with open(os.path.join(PROF, "c4_kernel_stats.csv")) as f:
        rows = [r for r in csv.DictReader(f) if rl["kernel"] in r["Name"]]
    assert rows, rl["kernel"]
    avg_ms = float(rows[0]["AverageNs"]) / 1e6
    assert abs(avg_ms - rl["launch_ms"]) / rl["launch_ms"] < 0.05
