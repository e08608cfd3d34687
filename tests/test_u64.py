"""GPU parity on the u64 edges of s2Model.Step, every engine forced.

main_test.go:313-343 (TestLargeSeqNumsNotTruncated) exists to catch tail /
match_seq_num truncation at 2^32; main.go:279 wraps the tail mod 2^64. The
checker has code regimes keyed on exactly these (csrc/history.cpp finalize):

  H_TAIL32   every reachable tail < 2^32 - 3: 32-bit tails, bounds and
             match_seq_nums in the packed kernels and the solo rounds
  H_NOWRAP   sum of num_records <= 2^63: 64-bit P1 bounds (search_kernel,
             the level search's grid rounds)
  wrap       P1 and P2 off
  +zh        a zero-record append with hashes: P2 off

Random concurrent histories over all of them (tests/helpers.py
random_history_u64: num_records independent of the hash count, tails near
2^32 - 4 .. 2^32 + 5, 2^63, 2^64 - k, match_seq_num = tail +- 2^32, tails
perturbed by +-2^32), through the event API (s2lc_history_from_events), are
checked against brute force and the WGL restatement with each engine forced
(auto / workgroup / workgroup-HBM / level) and the level search with and
without solo rounds / persistent rounds. H174's u64 variants (> 128 chains,
the level search) are checked against the committed reduced-search counts
(helpers.hard_variant) and, for the Illegal one, against oracle/reduced.c.
"""
import random

import pytest

import oracle as orc
import s2_verification_amd as s2
from helpers import (U64_REGIMES, config_digest, golden, hard_variant, random_history_u64, to_s2_events,
                     u64_regime)

pytestmark = pytest.mark.gpu

ENGINES = {"auto": s2.ENGINE_AUTO, "workgroup": s2.ENGINE_WORKGROUP, "workgroup_hbm": s2.ENGINE_WORKGROUP_HBM,
           "level": s2.ENGINE_LEVEL}
MODES = {"default": {}, "no_solo": {"S2LC_NO_SOLO": "1"}, "no_persist": {"S2LC_NO_PERSIST": "1"}}

_cases = {}


def _small_cases():
    """1,200 small histories (brute force = WGL), 300 per regime generator."""
    if "small" not in _cases:
        rng = random.Random(2024)
        evs, want = [], []
        for i in range(1200):
            ev = random_history_u64(rng, rng.randint(1, 9), n_clients=rng.randint(1, 4), regime=U64_REGIMES[i % 4])
            w, _ = orc.check_wgl(ev)
            assert orc.check_brute(ev)[0] == w
            evs.append(ev)
            want.append(w)
        _cases["small"] = (evs, want)
    return _cases["small"]


def _medium_cases():
    """240 histories of 14-30 ops over 3-6 clients (WGL within its timeout)."""
    if "medium" not in _cases:
        rng = random.Random(77)
        evs, want = [], []
        for i in range(300):
            ev = random_history_u64(rng, rng.randint(14, 30), n_clients=rng.randint(3, 6), regime=U64_REGIMES[i % 4],
                                    p_perturb=0.05)
            w, _ = orc.check_wgl(ev, timeout=10.0)
            if w == "Unknown":
                continue
            evs.append(ev)
            want.append(w)
            if len(evs) == 240:
                break
        _cases["medium"] = (evs, want)
    return _cases["medium"]


def _check(engine, evs, want, rc_check=False):
    hs = [s2.History.from_events(to_s2_events(ev)) for ev in evs]
    c = s2.Checker(engine=ENGINES[engine], round_counts=rc_check)
    b = c.batch(hs)
    res = b.check()
    bad = [(i, u64_regime(evs[i]), r.verdict, w) for i, (r, w) in enumerate(zip(res, want)) if r.verdict != w]
    assert not bad, (engine, bad[:8])
    for h, r in zip(hs, res):
        if r.verdict == s2.Ok:
            assert r.witness is not None and len(r.witness) == h.info()["n_ops"]
    return b, hs


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("engine", list(ENGINES))
def test_u64_small_vs_brute_and_wgl(engine, mode, monkeypatch):
    if mode != "default" and engine != "level":
        pytest.skip("solo / persistent rounds belong to the level search")
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    evs, want = _small_cases()
    regimes = {u64_regime(e).split("+")[0] for e in evs}
    assert regimes == {"tail32", "nowrap", "wrap"}
    b, _ = _check(engine, evs, want)
    if engine == "level":
        assert b.stats()["level_histories"] == len(evs)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("engine", list(ENGINES))
def test_u64_medium_vs_wgl(engine, mode, monkeypatch):
    if mode != "default" and engine != "level":
        pytest.skip("solo / persistent rounds belong to the level search")
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    evs, want = _medium_cases()
    assert {"Ok", "Illegal"} <= set(want)
    _check(engine, evs, want)


@pytest.mark.parametrize("engine", list(ENGINES))
def test_u64_round_counts_match_reduced_search(engine):
    """Per-round unique-configuration counts on the u64 histories equal
    oracle/reduced.c's (which take the same regime switches from the same
    sums): the regimes change which prunes run, never the configuration set
    the product and the CPU search agree on. (These cases found the one place
    where reduced.c and the engines had differed: an indefinite append whose
    guards fail and whose opt state equals its parent's, 0 records and no
    hashes; its identity child is deferred like any other.)"""
    evs, want = _small_cases()
    evs, want = evs + _medium_cases()[0], want + _medium_cases()[1]
    b, hs = _check(engine, evs, want, rc_check=True)
    for i, (ev, h) in enumerate(zip(evs, hs)):
        v, st = orc.check_reduced(ev, round_counts=True)
        assert v == want[i]
        assert b.round_counts(i) == st["round_counts"], (engine, i, u64_regime(ev))


def test_large_seq_nums_on_every_engine():
    """TestLargeSeqNumsNotTruncated (main_test.go:315-343) itself: tail
    2^32 + 5 from one append of NumRecords = 2^32 + 5 with a single hash, then
    an append guarded by match_seq_num 5 (Illegal) or 2^32 + 5 (Ok), through
    every engine."""
    def hist(msn):
        ev = [s2.Event(s2.CallEvent, s2.StreamInput(InputType=0, NumRecords=(1 << 32) + 5, RecordHashes=[7]), 0),
              s2.Event(s2.ReturnEvent, s2.StreamOutput(Tail=(1 << 32) + 5), 0),
              s2.Event(s2.CallEvent, s2.StreamInput(InputType=0, NumRecords=1, RecordHashes=[9], MatchSeqNum=msn), 1),
              s2.Event(s2.ReturnEvent, s2.StreamOutput(Tail=(1 << 32) + 6), 1)]
        return s2.History.from_events(ev)
    for engine in ENGINES.values():
        res = s2.Checker(engine=engine).check_many([hist(5), hist((1 << 32) + 5)])
        assert [r.verdict for r in res] == [s2.Illegal, s2.Ok], engine


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("variant", ["above32", "msn_exact", "zero_hash", "stale_msn"])
def test_h174_u64_variants(variant, mode, monkeypatch):
    """H174 (174 chains) with its u64 variants on the level search, in every
    round mode: above32 (64-bit tails: no solo rounds, the grid's 64-bit P1)
    and zero_hash (P2 off) against the committed counts transformed, msn_exact
    against H174's own counts, stale_msn (match_seq_num = pre-tail + 2^32 on
    one append, solo rounds under H_TAIL32) Illegal with the CPU reduced
    search's rounds and counts."""
    from s2_verification_amd import workloads as W
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    g = golden("hard_round_counts.json")["H174"]
    assert config_digest("H174") == g["digest"]
    hv = s2.History.from_events(hard_variant(W.config_history("H174").events(), variant))
    if variant == "stale_msn":
        v, st = orc.check_reduced(orc.from_s2lc_numpy(hv.events_numpy(), owner=hv), round_counts=True)
        assert v == s2.Illegal
        want = (v, st["rounds"], st["round_counts"])
    else:
        base = g["2" if variant == "zero_hash" else "0"]
        counts = ([1] if variant == "above32" else []) + base["counts"]
        want = (base["verdict"], len(counts), counts)
    c = s2.Checker(round_counts=True)
    b = c.batch([hv])
    r = b.check()[0]
    st = b.stats()
    assert (r.verdict, r.rounds, b.round_counts(0)) == want, (variant, mode, r, st)
    assert st["level_histories"] == 1
    if r.verdict == s2.Ok:
        assert r.witness is not None and len(r.witness) == hv.info()["n_ops"]
    if variant == "above32" or mode != "default":
        assert st["level_solo_rounds"] == 0, st
    else:
        assert st["level_solo_rounds"] > r.rounds // 2, st
