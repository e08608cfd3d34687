"""GPU parity of every search engine, forced route by route, and of the search
itself (per-round configuration counts) under reduction ablations.

The checker picks an engine per history (packed lane groups for K <= 32, one
workgroup per history for K <= 128, the device-wide level search above), so
the default route never sends the small parity cases through search_kernel.
Here the context forces each engine (s2lc_opts.engine) over the same cases:

  ENGINE_WORKGROUP      search_kernel, LDS pass then HBM-slab pass
  ENGINE_WORKGROUP_HBM  search_kernel, HBM-slab pass only
  ENGINE_LEVEL          lv_expand / lv_close / lv_insert

Round counts: with the same reductions on, the set of unique configurations
of every round is fixed (closure is canonical, dedupe exact), so the GPU's
count per completed round must equal oracle/reduced.c's. That pins the
search, not only the final verdict. Reductions are switched off one at a
time (s2lc_opts.reductions_off) on histories where the unreduced search stays
small; the hard histories are compared against committed counts
(tests/golden/hard_round_counts.json, tests/golden/make_round_counts.py).
"""
import os
import random
import subprocess

import pytest

import oracle as orc
import s2_verification_amd as s2
from helpers import GOLDEN, config_digest, from_s2_events, golden, random_history, to_s2_events

pytestmark = pytest.mark.gpu

ENGINES = {"auto": s2.ENGINE_AUTO, "workgroup": s2.ENGINE_WORKGROUP, "workgroup_hbm": s2.ENGINE_WORKGROUP_HBM,
           "level": s2.ENGINE_LEVEL}
_checkers = {}


def checker_for(engine=s2.ENGINE_AUTO, red=0, rc=False):
    key = (engine, red, rc)
    if key not in _checkers:
        _checkers[key] = s2.Checker(engine=engine, reductions_off=red, round_counts=rc)
    return _checkers[key]


def run(c, hs):
    b = c.batch(hs)
    res = b.check()
    return b, res


@pytest.mark.parametrize("engine", list(ENGINES))
def test_engine_reference_cases(engine):
    hs, expect = [], []
    for c in golden("reference_cases.json")["cases"]:
        hs.append(s2.History.from_events(to_s2_events(c["events"])))
        expect.append(c["expected"])
    _, res = run(checker_for(ENGINES[engine]), hs)
    for h, r, e in zip(hs, res, expect):
        assert r.verdict == e, (engine, r, e)
        if r.verdict == s2.Ok:
            assert r.witness is not None and len(r.witness) == h.info()["n_ops"]


@pytest.mark.parametrize("engine", list(ENGINES))
def test_engine_random_small_vs_brute_and_wgl(engine):
    rng = random.Random(7)
    hs, expect = [], []
    for _ in range(400):
        n = rng.randint(1, 9)
        ev = random_history(rng, n, n_clients=rng.randint(1, 4))
        b, _ = orc.check_brute(ev)
        w, _ = orc.check_wgl(ev)
        assert b == w
        hs.append(s2.History.from_events(to_s2_events(ev)))
        expect.append(w)
    bt, res = run(checker_for(ENGINES[engine]), hs)
    assert [r.verdict for r in res] == expect, engine
    assert all(r.witness is not None for r in res if r.verdict == s2.Ok)
    if engine == "level":
        assert bt.stats()["level_histories"] == len(hs)


@pytest.mark.parametrize("engine", ["workgroup", "workgroup_hbm", "level"])
@pytest.mark.parametrize("wf", [s2.WF_REGULAR, s2.WF_MATCH_SEQ_NUM, s2.WF_FENCING])
def test_engine_simulated_vs_wgl(engine, wf):
    viols = [s2.VIOL_NONE, s2.VIOL_READ_HASH, s2.VIOL_TAIL, s2.VIOL_DEFINITE_APPLIED, s2.VIOL_STALE_MSN]
    hs, expect = [], []
    for seed in range(30):
        h = s2.simulate_history(workflow=wf, num_clients=3 + seed % 4, ops_per_client=60, seed=1000 + seed,
                                violation=viols[seed % len(viols)], p_indefinite=0.03)
        w, _ = orc.check_wgl(from_s2_events(h.events()), timeout=20.0)
        if w == "Unknown":
            continue
        hs.append(h)
        expect.append(w)
    _, res = run(checker_for(ENGINES[engine]), hs)
    assert [r.verdict for r in res] == expect, (engine, wf)


@pytest.mark.parametrize("engine", ["workgroup", "workgroup_hbm", "level"])
def test_engine_c4_sample_vs_wgl(engine):
    from s2_verification_amd import workloads as W
    hs = W.c4_histories(300, first_seed=500)
    expect = [orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy()))[0] for h in hs]
    _, res = run(checker_for(ENGINES[engine]), hs)
    assert [r.verdict for r in res] == expect, engine
    assert all(r.witness is not None for r in res if r.verdict == s2.Ok)


@pytest.mark.parametrize("route", ["workgroup", "auto_many", "auto_few"])
@pytest.mark.parametrize("name", ["H48", "H48bad", "H96", "H100", "H120m"])
def test_mid_k_histories(name, route, monkeypatch):
    """32 < K <= 128 with the collector's client-id cap. The workgroup engine
    (search_kernel) forced, the default route of a batch with many of them
    (search_kernel: S2LC_MIDK_LEVEL_MAX=0 here), and of a batch with a few
    (the level search). Porcupine's DFS does not finish; verdict = the CPU
    reduced search."""
    from s2_verification_amd import workloads as W
    h = W.config_history(name)
    K = h.info()["n_chains"]
    assert 32 < K <= 128
    v, _ = orc.check_reduced(orc.from_s2lc_numpy(h.events_numpy(), owner=h))
    if route == "auto_many":
        monkeypatch.setenv("S2LC_MIDK_LEVEL_MAX", "0")
    ck = checker_for(s2.ENGINE_WORKGROUP) if route == "workgroup" else s2.Checker()
    b, res = run(ck, [h])
    r = res[0]
    st = b.stats()
    assert st["pack8_histories"] == 0 and st["pack16_histories"] == 0, st
    assert st["level_histories"] == (1 if route == "auto_few" else 0), st
    assert r.verdict == v, (name, r)
    if r.verdict == s2.Ok:
        assert r.witness is not None and len(r.witness) == h.info()["n_ops"]


@pytest.mark.parametrize("pack8", [True, False])
def test_packed_kernels_round_counts(pack8, monkeypatch):
    """The packed kernels (16-lane groups for K <= 16, or with S2LC_PACK8=1
    8-lane groups for K <= 8 first): verdicts and per-round unique-configuration
    counts equal the CPU reduced search."""
    from s2_verification_amd import workloads as W
    if pack8:
        monkeypatch.setenv("S2LC_PACK8", "1")
    hs = W.c4_histories(120, first_seed=8100) + [W.config_history(n) for n in ("C1", "C2", "C3")]
    c = s2.Checker(round_counts=True)
    b = c.batch(hs)
    res = b.check()
    st = b.stats()
    n8 = sum(1 for h in hs if h.info()["n_chains"] <= 8)
    assert (st["pack8_histories"] >= n8 - st["n_overflow"] and n8 > 0) if pack8 else st["pack8_histories"] == 0, st
    for i, (h, r) in enumerate(zip(hs, res)):
        v, ost = orc.check_reduced(orc.from_s2lc_numpy(h.events_numpy()), round_counts=True)
        assert r.verdict == v, (pack8, i, r, v)
        assert b.round_counts(i) == ost["round_counts"], (pack8, i)
        if r.verdict == s2.Ok:
            assert r.witness is not None and len(r.witness) == h.info()["n_ops"]


ABLATIONS = {"all_on": 0, "no_p1": s2.RED_P1, "no_p2": s2.RED_P2, "no_p4": s2.RED_P4, "no_idefer": s2.RED_IDEFER}
# histories whose search stays small with any one reduction off (oracle/reduced.c, this container: < 2 s each)
ROUND_CASES = ["C1", "C2", "C3", "H48", "H48bad", "H100", "H120m"]


def _round_cases():
    from s2_verification_amd import workloads as W
    hs = [W.config_history(n) for n in ROUND_CASES]
    hs += W.c4_histories(40, first_seed=7000)
    return hs


@pytest.mark.parametrize("engine", list(ENGINES))
@pytest.mark.parametrize("abl", list(ABLATIONS))
def test_round_counts_match_reduced_search(engine, abl):
    """Verdict and the unique-configuration count of every completed round
    equal the CPU reduced search with the same reductions switched off."""
    red = ABLATIONS[abl]
    hs = _round_cases()
    b, res = run(checker_for(ENGINES[engine], red, rc=True), hs)
    for i, (h, r) in enumerate(zip(hs, res)):
        v, st = orc.check_reduced(orc.from_s2lc_numpy(h.events_numpy()), reductions_off=red, round_counts=True)
        assert r.verdict == v, (engine, abl, i, r, v)
        assert r.rounds == st["rounds"], (engine, abl, i, r.rounds, st["rounds"])
        got = b.round_counts(i)
        assert got == st["round_counts"], (engine, abl, i, [k for k, (x, y) in enumerate(zip(got, st["round_counts"]))
                                                             if x != y][:5])


# level-search round modes: narrow rounds inside the persistent kernel, with
# one-configuration rounds as solo rounds of workgroup 0 (default) or on the
# grid (no_solo), host-enqueued rounds only (lv_round staging everything for
# lv_insert, or inserting as it expands: wide_fused), or every round inside
# the persistent kernel
LEVEL_MODES = {"default": {}, "no_solo": {"S2LC_NO_SOLO": "1"}, "no_persist": {"S2LC_NO_PERSIST": "1"},
               "wide_fused": {"S2LC_WIDE_FUSED": "1", "S2LC_NO_PERSIST": "1"},
               "all_persist": {"S2LC_PERSIST_NF": "4294967295"}}


def _set_mode(monkeypatch, mode):
    for k, v in LEVEL_MODES[mode].items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("mode", list(LEVEL_MODES))
@pytest.mark.parametrize("name,off", [("H174", 0), ("H174", 2), ("H212", 0), ("H212", 2), ("C5bad", 0),
                                      ("C5bad", 2), ("C5bad", 4), ("C5wide", 0)])
def test_hard_round_counts(name, off, mode, monkeypatch):
    """Hard single histories (> 128 chains, the level search): per-round counts
    against the committed CPU reduced-search counts, in every round mode."""
    from s2_verification_amd import workloads as W
    _set_mode(monkeypatch, mode)
    ref = golden("hard_round_counts.json")[name]
    assert config_digest(name) == ref["digest"], "simulator output changed: regenerate the fixture"
    want = ref[str(off)]
    h = W.config_history(name)
    b, res = run(checker_for(s2.ENGINE_AUTO, off, rc=True), [h])
    r = res[0]
    st = b.stats()
    assert r.verdict == want["verdict"], (name, off, mode, r)
    assert r.rounds == want["rounds"]
    got = b.round_counts(0)
    bad = [k for k, (x, y) in enumerate(zip(got, want["counts"])) if x != y]
    assert got == want["counts"], (name, off, mode, bad[:5])
    if r.verdict == s2.Ok:
        assert r.witness is not None
    if mode in ("no_persist", "wide_fused"):
        assert st["level_persist_rounds"] == 0, st
    else:
        assert st["level_persist_rounds"] > 0, st
    if mode == "all_persist":
        assert st["level_persist_rounds"] == r.rounds, st
    if mode in ("no_solo", "no_persist", "wide_fused"):
        assert st["level_solo_rounds"] == 0, st
    elif name != "C5wide":  # most rounds of these histories keep one configuration
        assert st["level_solo_rounds"] > r.rounds // 2, st


@pytest.mark.parametrize("mode", ["default", "no_persist"])
def test_level_buffers_grow_on_overflow(mode, monkeypatch):
    """The level search starts with a small staging capacity (here 16 MiB of
    buffers) and raises it when a round overflows: C5wide (frontier up to
    273 k) then gives the committed verdict and every round's count."""
    from s2_verification_amd import workloads as W
    _set_mode(monkeypatch, mode)
    monkeypatch.setenv("S2LC_LEVEL_BUDGET_MB", "16")
    ref = golden("hard_round_counts.json")["C5wide"]
    assert config_digest("C5wide") == ref["digest"]
    want = ref["0"]
    c = s2.Checker(round_counts=True)
    b = c.batch([W.config_history("C5wide")])
    r = b.check()[0]
    st = b.stats()
    assert r.verdict == want["verdict"] and r.rounds == want["rounds"], r
    assert b.round_counts(0) == want["counts"]
    assert st["level_grows"] >= 1, st
    assert r.witness is not None


@pytest.mark.parametrize("mode", ["default", "no_persist"])
@pytest.mark.parametrize("name,off", [("H174", 1), ("H174", 8), ("C5bad", 1), ("C5bad", 8)])
def test_hard_exploding_ablation_prefix(name, off, mode, monkeypatch):
    """P1 or the indefinite deferral switched off on the hard histories: the
    search explodes (tens of millions of configurations; make_round_counts.py),
    so the fixture holds the CPU reduced search's counts for every round it
    completed within a budget. Under a smaller budget the GPU must stop with
    Unknown (budget) and reproduce that prefix round by round."""
    from s2_verification_amd import workloads as W
    _set_mode(monkeypatch, mode)
    ref = golden("hard_round_counts.json")[name]
    assert config_digest(name) == ref["digest"], "simulator output changed: regenerate the fixture"
    want = ref[f"{off}p"]
    assert not want["complete"] and want["verdict"] == "Unknown"
    h = W.config_history(name)
    c = s2.Checker(round_counts=True, reductions_off=off, max_configs=2_000_000, engine=s2.ENGINE_LEVEL)
    b = c.batch([h])
    r = b.check(with_witness=False)[0]
    assert r.verdict == s2.Unknown and r.reason == "budget", r
    got = b.round_counts(0)
    assert 50 < len(got) < len(want["counts"]), (len(got), len(want["counts"]))
    bad = [k for k, (x, y) in enumerate(zip(got[:-1], want["counts"])) if x != y]
    assert not bad, (name, off, mode, bad[:5])


@pytest.mark.parametrize("mode", ["default", "no_solo", "no_persist"])
@pytest.mark.parametrize("name,off", [("A144", 0), ("A144", 1), ("A144", 2), ("A144", 4), ("A144", 8),
                                      ("A160", 0), ("A160", 2), ("A160", 8)])
def test_hard_complete_ablations(name, off, mode, monkeypatch):
    """Whole-search reduction ablations on > 128-chain histories (the level
    search): P1 off (A144, 4.9 M unique configurations) and the indefinite
    deferral off (A144, 36 k; A160, 4.2 M) run to the end on the CPU reduced
    search (make_round_counts.py). Verdict, round count and every round's
    unique-configuration count equal the committed fixture."""
    from s2_verification_amd import workloads as W
    _set_mode(monkeypatch, mode)
    ref = golden("hard_round_counts.json")[name]
    assert config_digest(name) == ref["digest"], "simulator output changed: regenerate the fixture"
    want = ref[str(off)]
    h = W.config_history(name)
    assert h.info()["n_chains"] > 128
    b, res = run(checker_for(s2.ENGINE_AUTO, off, rc=True), [h])
    r = res[0]
    assert r.verdict == want["verdict"], (name, off, mode, r)
    assert r.rounds == want["rounds"], (r.rounds, want["rounds"])
    got = b.round_counts(0)
    bad = [k for k, (x, y) in enumerate(zip(got, want["counts"])) if x != y]
    assert got == want["counts"], (name, off, mode, bad[:5])
    assert b.stats()["level_histories"] == 1
    if r.verdict == s2.Ok:
        assert r.witness is not None and len(r.witness) == h.info()["n_ops"]


@pytest.mark.parametrize("mode", ["default", "no_solo", "all_persist"])
@pytest.mark.parametrize("abl", ["all_on", "no_p2", "no_idefer"])
def test_level_persist_round_counts_match_reduced_search(mode, abl, monkeypatch):
    """The persistent rounds against oracle/reduced.c, round by round, on the
    small cases (level engine forced)."""
    _set_mode(monkeypatch, mode)
    red = ABLATIONS[abl]
    hs = _round_cases()
    b, res = run(checker_for(s2.ENGINE_LEVEL, red, rc=True), hs)
    for i, (h, r) in enumerate(zip(hs, res)):
        v, st = orc.check_reduced(orc.from_s2lc_numpy(h.events_numpy()), reductions_off=red, round_counts=True)
        assert r.verdict == v, (mode, abl, i, r, v)
        assert r.rounds == st["rounds"], (mode, abl, i, r.rounds, st["rounds"])
        assert b.round_counts(i) == st["round_counts"], (mode, abl, i)
        if r.verdict == s2.Ok:
            assert r.witness is not None


@pytest.mark.parametrize("mode", ["default", "all_persist"])
def test_level_staging_overflow_is_unknown_with_exact_prefix(mode, monkeypatch):
    """A staging array too small for H174's widest rounds (4,096 slots): the
    round that overflows (inside the persistent kernel or
    not) is re-run over frontier chunks, and when the round still does not fit
    the verdict is Unknown / frontier. Every round completed before it keeps
    the exact unique-configuration count of the CPU reduced search."""
    from s2_verification_amd import workloads as W
    _set_mode(monkeypatch, mode)
    monkeypatch.setenv("S2LC_LEVEL_SCAP", "4096")
    ref = golden("hard_round_counts.json")["H174"]["0"]
    h = W.config_history("H174")
    c = s2.Checker(round_counts=True)
    b = c.batch([h])
    r = b.check()[0]
    st = b.stats()
    assert r.verdict == s2.Unknown and r.reason == "frontier", (r, st)
    got = b.round_counts(0)
    assert 100 < len(got) < ref["rounds"]
    assert got[:-1] == ref["counts"][:len(got) - 1]  # the last (overflowing) round has no count
    assert st["level_chunk_retries"] > 0, st
    if mode == "all_persist":
        assert st["level_persist_rounds"] > 0, st


def test_rerun_does_not_reuse_stale_results(monkeypatch):
    """a batch run twice, where a level-search history ends in
    Unknown (frontier beyond capacity, forced small with S2LC_LEVEL_SCAP),
    must give the same results both times and never re-route that history
    through the workgroup passes."""
    from s2_verification_amd import workloads as W
    monkeypatch.setenv("S2LC_LEVEL_SCAP", "128")
    hs = [W.config_history("H174")] + W.c4_histories(50, first_seed=9000)
    c = s2.Checker()
    b = c.batch(hs)
    r1 = b.check()
    st1 = b.stats()
    r2 = b.check()
    st2 = b.stats()
    assert r1[0].verdict == s2.Unknown and r1[0].reason == "frontier", r1[0]
    # the overflowing history: same verdict and reason (where in the search the
    # tiny staging array overflows depends on which waves reserve slots first);
    # every other history: identical results
    assert (r1[0].verdict, r1[0].reason) == (r2[0].verdict, r2[0].reason)
    assert [(r.verdict, r.reason, r.configs_explored) for r in r1[1:]] == [(r.verdict, r.reason, r.configs_explored)
                                                                          for r in r2[1:]]
    assert st1["level_histories"] == st2["level_histories"] == 1
    assert st2["n_overflow"] == 0
    expect = [orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy()))[0] for h in hs[1:]]
    assert [r.verdict for r in r2[1:]] == expect


def test_timeout_gives_unknown():
    """CheckEventsVerbose's timeout (main.go:606 passes 0): past it, Unknown."""
    from s2_verification_amd import workloads as W
    h = W.config_history("C5")  # ~0.5 s of level search
    r = s2.Checker(timeout=0.005).check(h)
    assert r.verdict == s2.Unknown and r.reason == "timeout", r
    hs = W.c4_histories(200)
    res = s2.Checker(timeout=1e-6).check_many(hs)
    assert all(r.verdict in (s2.Unknown, s2.Ok, s2.Illegal) for r in res)
    assert any(r.reason == "timeout" for r in res)
    # no timeout: decided
    res = s2.Checker(timeout=60).check_many(hs)
    assert all(r.verdict != s2.Unknown for r in res)
    v, info = s2.check_events_verbose(None, h, timeout=0.005)
    assert v == s2.Unknown


def test_timeout_ends_the_level_search_inside_its_launch():
    """The run's deadline is checked inside lv_persist (every grid round, every
    16 solo rounds), not only by the host between launches of up to 4,096
    rounds: a C5 (solo rounds) or C5wide (grid rounds) search with a short
    timeout returns Unknown (timeout) within a few milliseconds of it."""
    import time
    from s2_verification_amd import workloads as W
    for name, tmo in (("C5", 0.02), ("C5wide", 0.008)):
        h = W.config_history(name)
        ck = s2.Checker(timeout=tmo)
        ck.check(h)  # (warm: runtime, code objects, level buffers)
        t = time.perf_counter()
        r = ck.check(h)
        dt = time.perf_counter() - t
        assert r.verdict == s2.Unknown and r.reason == "timeout", (name, r)
        assert dt < tmo + 0.015, (name, dt)


def test_witness_certificate_failure_is_loud(monkeypatch, tmp_path):
    """an Ok whose witness fails CPU replay must not pass as Ok
    (test hook S2LC_FAULT_WITNESS corrupts every witness before certification)."""
    from s2_verification_amd import workloads as W
    monkeypatch.setenv("S2LC_FAULT_WITNESS", "1")
    c = s2.Checker()
    h = W.config_history("C1")
    with pytest.raises(s2.S2LCError) as e:
        c.check(h)
    assert e.value.status == s2.EWITNESS
    b = c.batch(W.c4_histories(20))
    b.run()
    with pytest.raises(s2.S2LCError) as e:
        b.results(with_witness=True)
    assert e.value.status == s2.EWITNESS
    assert all(r.verdict != s2.Unknown for r in b.results(with_witness=False))
    p = subprocess.run([s2.CLI_PATH, "-file=" + os.path.join(GOLDEN, "ref_BasicNoConcurrency.jsonl")],
                       capture_output=True, text=True, timeout=120, cwd=tmp_path, env=dict(os.environ))
    assert p.returncode == 3 and "failed: witness certification" in p.stderr, p.stderr


def test_multi_device_sharded_check_batch():
    """s2lc_opts.devices: LPT placement over shards (two shards on this one GPU),
    verdicts gathered in input order, equal to the single-shard run."""
    from s2_verification_amd import workloads as W
    hs = W.c4_histories(300, first_seed=1234) + [W.config_history("C2"), W.config_history("H48")]
    one = s2.Checker().check_many(hs)
    two = s2.Checker(devices=[0, 0]).check_many(hs)
    three = s2.Checker(devices=[0, 0, 0]).check_many(hs, as_numpy=True)
    assert [r.verdict for r in one] == [r.verdict for r in two] == [r.verdict for r in three]
    assert [r.configs_explored for r in one] == [r.configs_explored for r in two]
    for a, c in zip(one, three):
        assert (a.witness is None) == (c.witness is None)
        if a.witness is not None:
            assert list(c.witness) == a.witness


def test_device_fold_known_answers():
    """foldRecordHashes on the device (the search kernels' routine) against the
    reference vectors (main_test.go:15-32) and the python-xxhash golden pairs."""
    g = golden("chain_hash_vectors.json")
    c = s2.Checker()
    seeds = [h for h, _, _ in g["pairs"]] + [h for h, _, _ in g["folds"]]
    folds = [[r] for _, r, _ in g["pairs"]] + [list(rs) for _, rs, _ in g["folds"]]
    want = [w for _, _, w in g["pairs"]] + [w for _, _, w in g["folds"]]
    assert len(g["pairs"]) >= 449 and len(g["folds"]) >= 40
    assert c.device_fold(seeds, folds) == want
    # chain over foo, bar, baz from seed 0 (main_test.go:15-32)
    ref = g["reference"]
    x = ref["xxh3"]
    assert c.device_fold([0, 0, 0], [x[:1], x[:2], x]) == [ref["h1"], ref["h2"], ref["h3"]]


def test_check_reuses_scratch_and_matches_batch():
    """s2lc_check through the context's scratch batch, called repeatedly with
    histories of growing and shrinking size, gives the batch path's verdicts."""
    from s2_verification_amd import workloads as W
    c = s2.Checker()
    hs = [W.config_history(n) for n in ("C1", "C3", "C2", "H48", "C1")] + W.c4_histories(20)
    want = [r.verdict for r in s2.Checker().check_batch(hs)]
    got = [c.check(h).verdict for h in hs]
    assert got == want


def test_results_flat_matches_results():
    """s2lc_batch_results_flat: the same verdicts, counts and certified
    witnesses as s2lc_batch_results, as flat arrays."""
    from s2_verification_amd import workloads as W
    import numpy as np
    hs = W.c4_histories(300, first_seed=4200) + [W.config_history("C3")]
    c = s2.Checker()
    b = c.batch(hs)
    b.run()
    res = b.results(with_witness=True)
    flat = b.results_flat(with_witness=True)
    offs = flat["witness_offs"].astype(np.int64)
    assert offs[-1] == len(flat["witness_ids"])
    for i, r in enumerate(res):
        assert s2._VERDICT[int(flat["verdict"][i])] == r.verdict
        assert int(flat["configs"][i]) == r.configs_explored and int(flat["rounds"][i]) == r.rounds
        w = flat["witness_ids"][offs[i]:offs[i + 1]].tolist()
        assert w == (list(r.witness) if r.verdict == s2.Ok else []), i
    assert any(r.verdict == s2.Illegal for r in res) and any(r.verdict == s2.Ok for r in res)
    nw = b.results_flat(with_witness=False)
    assert (nw["witness_offs"] == 0).all() and (nw["verdict"] == flat["verdict"]).all()


@pytest.mark.parametrize("plain", [False, True])
def test_persist_fallback_keeps_round_counts(plain, monkeypatch):
    """ADVICE / VERDICT r2: lv_persist's grid barrier. A barrier wait past its
    limit (forced here: 1 us, so the first wait of a launch gives up) must not
    surface as an error: the search restarts from round 0 with host-driven
    rounds, with the same verdict and the same unique-configuration count in
    every round as the committed CPU reduced search. Cooperative launches and
    plain ones (S2LC_PERSIST_PLAIN=1)."""
    from s2_verification_amd import workloads as W
    monkeypatch.setenv("S2LC_PERSIST_SPIN_US", "1")
    if plain:
        monkeypatch.setenv("S2LC_PERSIST_PLAIN", "1")
    ref = golden("hard_round_counts.json")["H174"]
    want = ref["0"]
    h = W.config_history("H174")
    c = s2.Checker(round_counts=True)
    b = c.batch([h])
    r = b.check()[0]
    st = b.stats()
    assert r.verdict == want["verdict"] and r.rounds == want["rounds"], (r, st)
    assert b.round_counts(0) == want["counts"]
    assert st["level_persist_fallbacks"] == 1 and st["level_solo_rounds"] == 0, st
    if r.verdict == s2.Ok:
        assert r.witness is not None and len(r.witness) == h.info()["n_ops"]
    # the same batch's next search runs host-driven from the start (the
    # fallback is sticky per device batch: no further persistent launch)
    r1 = b.check()[0]
    st1 = b.stats()
    assert (r1.verdict, r1.rounds) == (r.verdict, r.rounds) and b.round_counts(0) == want["counts"]
    assert st1["level_persist_launches"] == 0 and st1["level_persist_fallbacks"] == 0, st1


def test_concurrent_contexts_persistent_rounds():
    """Two contexts on GPU 0 checking hard histories from two threads at once
    (each with persistent grids of 256 workgroups), and one context sharding
    H174 + H212 over devices=[0, 0]: verdicts and round counts as committed."""
    import threading
    from s2_verification_amd import workloads as W
    rc = golden("hard_round_counts.json")
    names = ["H174", "H212"]
    hs = {n: W.config_history(n) for n in names}
    out, errs = {}, []

    def work(name):
        try:
            c = s2.Checker(round_counts=True)
            b = c.batch([hs[name]])
            r = b.check()[0]
            out[name] = (r.verdict, r.rounds, b.round_counts(0), r.witness is not None, b.stats())
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(n,)) for n in names]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    for n in names:
        v, rounds, counts, has_w, st = out[n]
        want = rc[n]["0"]
        assert (v, rounds) == (want["verdict"], want["rounds"]), (n, v, rounds, st)
        assert counts == want["counts"], n
        assert v != s2.Ok or has_w
    res = s2.Checker(devices=[0, 0]).check_many([hs["H174"], hs["H212"]])
    assert [r.verdict for r in res] == [rc[n]["0"]["verdict"] for n in names]
    assert [r.rounds for r in res] == [rc[n]["0"]["rounds"] for n in names]


@pytest.mark.parametrize("mode", ["default", "no_solo", "no_persist"])
def test_budget_inside_a_one_configuration_stretch(mode, monkeypatch):
    """The configuration budget trips inside a stretch of one-configuration
    rounds (H174 round 5,000 of 10,285; the solo rounds close such rounds on
    registers and hold the budget as a count of rounds left): Unknown (budget)
    at the same round in every mapping, one round later per configuration of
    budget, with the committed counts before it."""
    from s2_verification_amd import workloads as W
    _set_mode(monkeypatch, mode)
    ref = golden("hard_round_counts.json")["H174"]
    assert config_digest("H174") == ref["digest"], "simulator output changed: regenerate the fixture"
    want = ref["0"]["counts"]
    r = next(i for i in range(5000, len(want) - 20) if all(c == 1 for c in want[i - 20:i + 20]))
    cum = sum(want[:r + 1])
    h = W.config_history("H174")
    for extra in (0, 1, 2):
        c = s2.Checker(round_counts=True, max_configs=cum - 1 + extra, engine=s2.ENGINE_LEVEL)
        b = c.batch([h])
        res = b.check(with_witness=False)[0]
        assert res.verdict == s2.Unknown and res.reason == "budget", (extra, res)
        got = b.round_counts(0)
        assert res.rounds == r + extra and len(got) == r + extra, (extra, res.rounds, len(got), r)
        assert got == want[:len(got)], extra
