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


@pytest.mark.gpu
def test_bench_two_gloo_ranks_on_one_gpu():
    """The driver's multi-GPU bench path, rehearsed with 2 ranks sharing the one
    GPU over gloo (S2LC_BENCH_GLOO=1): the weak C4 line, the strong split of
    the BASELINE C4 batch (10,000 histories in total: the committed CPU
    verdict counts), and the distributed C5 / C5wide legs (verdicts against
    the committed reduced search, witnesses certified)."""
    import random
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import golden
    port = random.randint(20000, 40000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-e2e", "--c5-reps", "1"]
    env = dict(os.environ, S2LC_BENCH_GLOO="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["verdicts"]["Unknown"] == 0
    c4 = golden("c4_verdicts.json")
    ss = d["strong_split"]
    assert ss["histories_total"] == 10000 and ss["histories_per_gpu"] == 5000
    assert ss["verdicts"] == {"Ok": sum(1 for r in c4["rows"] if r[0] == "O"),
                              "Illegal": sum(1 for r in c4["rows"] if r[0] == "I"), "Unknown": 0}
    hard = golden("hard_reduced.json")
    c5 = d["c5"]
    assert "error" not in c5, c5
    assert c5["verdict"] == hard["C5"]["verdict"] and c5["witness_replayed"], c5
    assert c5["bad_variant_verdict"] == hard["C5bad"]["verdict"]
    assert c5["replicated_only"]["verdict"] == c5["verdict"]
    # every rank self-checks H212 / C5bad with forced block
    # overflows and re-runs before the timed C5 legs
    dp = d["dist_parity"]
    assert dp["ok"] is True and dp["failing_cases_summed_over_ranks"] == 0, dp
    for name in ("H212", "C5bad"):
        cs = dp["cases"][name]
        assert cs["verdict"] == hard[name]["verdict"] and cs["rounds"] == hard[name]["reduced"]["rounds"], cs
        assert cs["xreruns_rank0"] >= 1 and cs["partitioned_rounds"] > 0, cs
    assert d["config"]["client_id_cap"] == 20 and c5["client_id_cap"] > 20 and c5["n_ops_planned"] == 32000
    w = c5["c5wide"]
    assert w["verdict"] == hard["C5wide"]["verdict"] and w["witness_replayed"], w
    # the N-GPU legs carry the single-GPU engine's time and the
    # speed-up against it (not against the replicated-only distributed path)
    for leg, name in ((c5, "C5"), (w, "C5wide")):
        assert leg["single_gpu_verdict"] == hard[name]["verdict"], (name, leg)
        assert leg["single_gpu_seconds"] > 0 and leg["speedup"] > 0, (name, leg)
        assert abs(leg["speedup"] - leg["single_gpu_seconds"] / leg["seconds"]) < 0.01 * leg["speedup"] + 1e-3


@pytest.mark.gpu
def test_bench_watchdog_keeps_the_c4_line():
    """A multi-GPU leg that stalls must not cost the C4 line, and must not read
    as success: with a watchdog budget far below the legs' time,
    every rank ends itself and rank 0 prints the line with the legs finished
    so far (the C4 measurement), `stalled_leg` and a `watchdog` note; the run
    exits non-zero."""
    import random
    port = random.randint(20000, 40000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-e2e", "--c5-reps", "1"]
    env = dict(os.environ, S2LC_BENCH_GLOO="1", S2LC_BENCH_WATCHDOG="0.05")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode != 0, p.stdout[-2000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert "watchdog" in d and d["n_gpus"] == 2 and d["value"] > 0 and d["verdicts"]["Unknown"] == 0, d
    assert d["stalled_leg"] == "strong_split" and "strong_split" not in d and "c5" not in d, d
