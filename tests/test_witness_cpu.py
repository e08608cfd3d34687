"""Witness rebuild + CPU-model certification (csrc/witness.cpp) without a GPU.

tests/witness_bench/bench.cpp finds a move list for each of the first C4-style
simulator histories with a small CPU breadth-first search (the device search's
rounds with its E-closure), then certifies each through s2lc_witness_from_moves
and checks that broken move lists (an unknown chain first, the last move
dropped) are rejected. The digest of the certified witnesses (op ids in order)
is pinned: it is the value the certifier produced on the same histories
before the round-6 closure rework (commit 8b7c0a2, built from its sources and
compared here; on the GPU the rework was compared on the 10k C4 batch,
profiles/r06/cert/).
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "s2_verification_amd")
N_HIST = 120
DIGEST = "9d1d4f3561ab39f7"


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libs2lincheck.so")):
        pytest.skip("libs2lincheck.so not built")
    out = str(tmp_path_factory.mktemp("wb") / "bench")
    cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(LIBDIR, "csrc"), os.path.join(ROOT, "tests", "witness_bench", "bench.cpp"),
           "-o", out, "-L" + LIBDIR, "-ls2lincheck", "-Wl,-rpath," + LIBDIR]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return out


def test_certified_witnesses_and_rejections(harness):
    r = subprocess.run([harness, str(N_HIST)], capture_output=True, text=True, timeout=600)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    by = {k: v for d in lines for k, v in d.items()}
    assert r.returncode == 0, r.stdout + r.stderr
    assert by["histories"] == N_HIST and by["failed"] == 0
    assert by["negatives"] > 0 and by["rejected"] == by["negatives"]
    assert by["witness_digest"] == DIGEST
