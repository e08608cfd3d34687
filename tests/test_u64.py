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
from helpers import (U64_REGIMES, _fold, config_digest, golden, hard_variant, random_history_u64, to_s2_events,
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


def _small_edge_cases():
    """~600 small histories around the 16-bit fields of the 32-byte records
    (regime "small_edge"), brute force = WGL, split by whether the host packs
    them as H_SMALL (every append's num_records summed <= 65,532)."""
    if "small_edge" not in _cases:
        rng = random.Random(65532)
        sm, big = ([], []), ([], [])
        for _ in range(600):
            ev = random_history_u64(rng, rng.randint(1, 9), n_clients=rng.randint(1, 4), regime="small_edge")
            w, _ = orc.check_wgl(ev)
            assert orc.check_brute(ev)[0] == w
            tot = sum(min(e["num_records"], 1 << 32) for e in ev if e["kind"] == "call" and e["input_type"] == 0)
            dst = sm if tot <= 65532 else big
            dst[0].append(ev)
            dst[1].append(w)
        _cases["small_edge"] = (sm, big)
    return _cases["small_edge"]


def _sequential_appends(n_ops, bad_last):
    """One client, n_ops appends of one record in a row (tails 1..n_ops); the
    last return off by one when bad_last."""
    evs = []
    for i in range(n_ops):
        evs.append(s2.Event(s2.CallEvent, s2.StreamInput(InputType=0, NumRecords=1, RecordHashes=[]), i, 0))
        evs.append(s2.Event(s2.ReturnEvent, s2.StreamOutput(Tail=i + 1 + (1 if bad_last and i == n_ops - 1 else 0)),
                            i, 0))
    return s2.History.from_events(evs)


def _hash_count_history(n_hashes, bad):
    """An append of n_hashes record hashes, then a read of the folded hash
    (a bit flipped when bad): oracle dict events."""
    rng = random.Random(n_hashes)
    hs = [rng.getrandbits(64) for _ in range(n_hashes)]
    ev = [{"kind": "call", "op_id": 0, "client_id": 0, "input_type": 0, "num_records": 2, "record_hashes": hs,
           "set_fencing_token": None, "fencing_token": None, "match_seq_num": None},
          {"kind": "return", "op_id": 0, "client_id": 0, "failure": False, "definite_failure": False, "tail": 2,
           "stream_hash": None},
          {"kind": "call", "op_id": 1, "client_id": 1, "input_type": 1},
          {"kind": "return", "op_id": 1, "client_id": 1, "failure": False, "definite_failure": False, "tail": 2,
           "stream_hash": None}]
    ev[3]["stream_hash"] = _fold(0, hs) ^ (1 if bad else 0)
    return ev


@pytest.mark.parametrize("small", ["1", "0"])
def test_small_records_at_their_bounds(small, monkeypatch):
    """The packed kernels' 32-byte records (csrc/search.h SRec: 16-bit
    num_records, match_seq_num, tails, event indices and hash counts,
    saturating) against brute force / WGL at their bounds: random histories
    whose tails end at 65,520 .. 65,537 with match_seq_num = tail +- 2^16 and
    0xFFFD .. 0x10000 (a batch of H_SMALL histories and a batch of the rest),
    65,534 / 65,536 events, 65,535 / 65,536 hashes on one append. With
    S2LC_PACK_SMALL=0 every list takes the 64-byte records: same verdicts."""
    monkeypatch.setenv("S2LC_PACK_SMALL", small)
    sm, big = _small_edge_cases()
    assert len(sm[0]) > 100 and len(big[0]) > 100 and {"Ok", "Illegal"} <= set(sm[1]) and {"Ok", "Illegal"} <= set(big[1])
    b, _ = _check("auto", *sm)
    st = b.stats()
    assert st["pack16_histories"] == len(sm[0]), st
    assert st["pack16_small"] == (len(sm[0]) if small == "1" else 0), st
    b, _ = _check("auto", *big)
    assert b.stats()["pack16_small"] == 0
    # the other engines read the 64-byte records widened on the device from
    # the uploaded 32-byte ones (search.h from_srec)
    for engine in ("workgroup", "level"):
        _check(engine, *sm)
    # event indices: 65,534 events fit (0xFFFF is "never"), 65,536 do not
    for n_ops, want_small in ((32767, True), (32768, False)):
        hs = [_sequential_appends(n_ops, False), _sequential_appends(n_ops, True)]
        b = s2.Checker().batch(hs)
        assert [r.verdict for r in b.check()] == [s2.Ok, s2.Illegal]
        assert b.stats()["pack16_small"] == (2 if want_small and small == "1" else 0), (n_ops, b.stats())
    # hash counts: 65,535 fit in the 16-bit count, 65,536 do not
    for n, want_small in ((65535, True), (65536, False)):
        evs = [_hash_count_history(n, False), _hash_count_history(n, True)]
        assert [orc.check_wgl(ev)[0] for ev in evs] == [s2.Ok, s2.Illegal]
        b, _ = _check("auto", evs, [s2.Ok, s2.Illegal])
        assert b.stats()["pack16_small"] == (2 if want_small and small == "1" else 0), (n, b.stats())


@pytest.mark.parametrize("small", ["1", "0"])
def test_small_records_in_sliced_uploads(small, monkeypatch):
    """Batches of >= 2,048 histories are packed and uploaded in 16 slices,
    each slice's records as SRec (H_SMALL histories) and / or OpRec (the
    rest). A batch mixing both (2,400 histories, the small_edge cases four
    times, interleaved) runs the packed kernels' 64-byte instance, which reads
    the small histories' widened records; an all-small batch runs the 32-byte
    instance. Verdicts against brute force / WGL, every engine forced."""
    monkeypatch.setenv("S2LC_PACK_SMALL", small)
    sm, big = _small_edge_cases()
    evs, want = [], []
    for _ in range(4):
        for i in range(max(len(sm[0]), len(big[0]))):
            for src in (sm, big):
                if i < len(src[0]):
                    evs.append(src[0][i])
                    want.append(src[1][i])
    assert len(evs) >= 2048
    for engine in ("auto", "workgroup", "level"):
        b, _ = _check(engine, evs, want)
        if engine == "auto":
            assert b.stats()["pack16_small"] == 0
    evs_s, want_s = sm[0] * 6, sm[1] * 6
    b, _ = _check("auto", evs_s, want_s)
    assert b.stats()["pack16_small"] == (len(evs_s) if small == "1" else 0)
