"""CPU: s2-porcupine CLI surface that does not reach the checker (main.go:568-603)."""
import os
import subprocess

import s2_verification_amd as s2
from helpers import GOLDEN


def run(*args, stdin=None):
    return subprocess.run([s2.CLI_PATH, *args], capture_output=True, text=True, timeout=60, input=stdin)


def test_version():
    p = run("-version")
    assert p.returncode == 0 and p.stdout.startswith("s2-porcupine version ")


def test_usage_without_file():
    p = run()
    assert p.returncode == 1 and "usage:" in p.stderr and "-file=records-<epoch>.jsonl" in p.stderr


def test_open_error():
    p = run("-file=/nonexistent/records.jsonl")
    assert p.returncode == 1 and '"msg":"open file"' in p.stderr and '"level":"ERROR"' in p.stderr


def test_decode_error_before_device():
    p = run("-file", "-", stdin='{"event":{"Start":"Read"},"client_id":1,"op_id":1')
    assert p.returncode == 1 and p.stderr.startswith("failed to decode history:")
    p = run("-file=" + os.path.join(GOLDEN, "make_golden.py"))
    assert p.returncode == 1 and "failed to decode history" in p.stderr


def test_simulator_cli_matches_library(tmp_path):
    """s2-simulate (collect-history.rs arguments) writes ./data/records.<epoch>.jsonl,
    prints its path, and the bytes equal s2lc_simulate_jsonl for the same parameters."""
    exe = os.path.join(os.path.dirname(s2.CLI_PATH), "s2-simulate")
    p = subprocess.run([exe, "basin", "stream", "--num-concurrent-clients", "4", "--num-ops-per-client", "30",
                        "--workflow", "fencing", "--seed", "11", "--violation", "tail"],
                       capture_output=True, text=True, timeout=60, cwd=tmp_path)
    assert p.returncode == 0, p.stderr
    path = p.stdout.strip()
    assert path.startswith("./data/records.") and path.endswith(".jsonl")
    data = (tmp_path / path).read_bytes()
    want = s2.simulate_jsonl(workflow=s2.WF_FENCING, num_clients=4, ops_per_client=30, seed=11,
                             violation=s2.VIOL_TAIL)
    assert data == want
    h = s2.events_from_reader(data)  # the loader accepts it
    assert h.info()["n_ops"] > 0
    bad = subprocess.run([exe, "basin"], capture_output=True, text=True, timeout=60, cwd=tmp_path)
    assert bad.returncode == 2 and "usage" in bad.stderr
