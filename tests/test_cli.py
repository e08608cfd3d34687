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
