"""The C ABI from a plain C99 caller (tests/c_abi/cgo_sequence.c): the exact
call sequence of the Go cgo shim in INTEGRATION.md §2. Compiled with gcc
-std=c99 -pedantic -Werror against include/s2lincheck.h and linked against
the in-tree libs2lincheck.so."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "s2_verification_amd")


def build(tmp_path):
    exe = str(tmp_path / "cgo_sequence")
    cmd = ["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c_abi", "cgo_sequence.c"), "-o", exe, "-L", LIBDIR, "-ls2lincheck",
           "-Wl,-rpath," + LIBDIR]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return exe


def test_c99_caller_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: test_c99_caller_on_gpu covers the full sequence")
    exe = build(tmp_path)
    p = subprocess.run([exe, "--no-gpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all checks passed (no-gpu)" in p.stdout


@pytest.mark.gpu
def test_c99_caller_on_gpu(tmp_path):
    exe = build(tmp_path)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all checks passed (gpu)" in p.stdout
