"""GPU parity of the device-wide level search (csrc/level_dev.h).

Two ways in:
  * S2LC_LEVEL_ONLY=1 routes EVERY history of a batch through the level search,
    so the small-history parity cases (brute force / porcupine WGL restatement)
    exercise it directly;
  * histories with more than 128 chains always take it: the hard single
    histories of workloads.CONFIGS, checked against the CPU reduced search's
    verdicts committed in tests/golden/hard_reduced.json (made by
    tests/golden/make_hard_golden.py), every Ok witness replayed through the
    CPU model.
"""
import random

import pytest

import oracle as orc
import s2_verification_amd as s2
from helpers import golden, config_digest, random_history, to_s2_events

pytestmark = pytest.mark.gpu


@pytest.fixture
def level_only(monkeypatch):
    monkeypatch.setenv("S2LC_LEVEL_ONLY", "1")
    yield


def test_level_reference_cases(checker, level_only):
    hs, expect = [], []
    for c in golden("reference_cases.json")["cases"]:
        hs.append(s2.History.from_events(to_s2_events(c["events"])))
        expect.append(c["expected"])
    b = checker.batch(hs)
    res = b.check()
    assert b.stats()["level_histories"] == len([h for h in hs if h.info()["structural"] == 0])
    for h, r, e in zip(hs, res, expect):
        assert r.verdict == e, (r, e)
        if r.verdict == s2.Ok:
            assert r.witness is not None and len(r.witness) == h.info()["n_ops"]


def test_level_random_small_vs_brute(checker, level_only):
    rng = random.Random(11)
    hs, expect = [], []
    for _ in range(300):
        n = rng.randint(1, 9)
        ev = random_history(rng, n, n_clients=rng.randint(1, 4))
        b, _ = orc.check_brute(ev)
        hs.append(s2.History.from_events(to_s2_events(ev)))
        expect.append(b)
    res = checker.check_batch(hs)
    for i, (r, e) in enumerate(zip(res, expect)):
        assert r.verdict == e, (i, r, e)
        if r.verdict == s2.Ok:
            assert r.witness is not None


def test_level_c4_sample_vs_wgl(checker, level_only):
    from s2_verification_amd import workloads as W
    hs = W.c4_histories(200, first_seed=3000)
    expect = [orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy()))[0] for h in hs]
    res = checker.check_batch(hs)
    assert [r.verdict for r in res] == expect
    assert all(r.witness is not None for r in res if r.verdict == s2.Ok)


def test_level_configs_c1_c3(checker, level_only):
    from s2_verification_amd import workloads as W
    for name in ("C1", "C2", "C3"):
        h = W.config_history(name)
        r_, st = orc.check_reduced(orc.from_s2lc_numpy(h.events_numpy()))
        g = checker.check(h)
        assert g.verdict == r_, (name, g, r_)
        # same reductions => same number of unique configurations (Ok stops at the
        # first completing child, so only the rounds before it are comparable)
        if g.verdict == s2.Ok:
            assert g.witness is not None and len(g.witness) == h.info()["n_ops"]


@pytest.mark.parametrize("name", ["H174", "H212", "C5bad", "C5", "C5wide"])
def test_hard_single_history(checker, name):
    """> 128 chains: always the level search. Verdict = CPU reduced search
    (committed), Ok witness replay-verified; the bad C5 differs from C5 in
    exactly one ReadSuccess stream hash."""
    from s2_verification_amd import workloads as W
    ref = golden("hard_reduced.json")
    if name not in ref:
        pytest.skip(f"{name}: no committed reduced-search verdict")
    h = W.config_history(name)
    assert config_digest(name) == ref[name]["digest"], "simulator output changed: regenerate the fixture"
    assert h.info()["n_chains"] > 128
    b = checker.batch([h])
    r = b.check()[0]
    st = b.stats()
    assert st["level_histories"] == 1
    assert r.verdict == ref[name]["verdict"], (name, r, st)
    if r.verdict == s2.Ok:
        assert r.witness is not None and len(r.witness) == h.info()["n_ops"]


@pytest.mark.parametrize("mode", [{}, {"S2LC_NO_SOLO": "1"}, {"S2LC_NO_PERSIST": "1"}])
def test_dedupe_under_forced_tag_collisions(mode, monkeypatch):
    """The level search's dedupe tables compare the whole configuration on a
    tag hit and probe on. S2LC_TAG_DROP clears all but 8 bits of every tag and
    first slot (256 of each), so distinct configurations meet on one tag all
    the time: H174 must still give the committed reduced-search round counts
    (every unique configuration kept, every duplicate dropped) in each round
    mode: solo + persistent grid rounds (batched inserts), grid rounds only,
    host-enqueued rounds (lv_insert)."""
    from s2_verification_amd import workloads as W
    monkeypatch.setenv("S2LC_TAG_DROP", "0xFFFFFF00")
    for k, v in mode.items():
        monkeypatch.setenv(k, v)
    g = golden("hard_round_counts.json")["H174"]
    assert config_digest("H174") == g["digest"]
    h = W.config_history("H174")
    b = s2.Checker(round_counts=True).batch([h])
    r = b.check()[0]
    assert (r.verdict, b.round_counts(0)) == (g["0"]["verdict"], g["0"]["counts"]), (mode, r)
    assert r.witness is not None and len(r.witness) == h.info()["n_ops"]
