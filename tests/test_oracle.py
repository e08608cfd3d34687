"""CPU: the oracle (restatement of the reference) pinned against golden fixtures."""
import random

import oracle as orc
from helpers import golden, random_history


def test_chain_hash_reference_vectors():
    """TestChainHashVectors (main_test.go:15-32) / chain_hash_vectors (history.rs:678-687)."""
    g = golden("chain_hash_vectors.json")["reference"]
    foo, bar, baz = g["xxh3"]
    assert foo == 0xab6e5f64077e7d8a
    h1 = orc.chain_hash(0, foo)
    h2 = orc.chain_hash(h1, bar)
    h3 = orc.chain_hash(h2, baz)
    assert (h1, h2, h3) == (0x4d2b003ee417c3a5, 0x132e5d5dd7936edd, 0x732ee99abc5002ff)


def test_chain_hash_xxhash_vectors():
    g = golden("chain_hash_vectors.json")
    for h, r, want in g["pairs"]:
        assert orc.chain_hash(h, r) == want
    for h, rs, want in g["folds"]:
        assert orc.fold(h, rs) == want


def test_reference_verdict_cases():
    """The reference's 9 verdict tests + the large-line test, as fixtures."""
    for c in golden("reference_cases.json")["cases"]:
        v, _ = orc.check_wgl(c["events"])
        assert v == c["expected"], c["name"]
        b, _ = orc.check_brute(c["events"])
        assert b == c["expected"], c["name"]


def test_reference_jsonl_fixtures_decode_like_events():
    import os
    from helpers import GOLDEN
    for c in golden("reference_cases.json")["cases"]:
        if not c.get("jsonl_file"):
            continue
        with open(os.path.join(GOLDEN, c["jsonl_file"])) as f:
            ev = orc.load_jsonl(f.read())
        assert orc.check_wgl(ev)[0] == c["expected"]


def test_wgl_matches_brute_force_on_random_histories():
    rng = random.Random(12345)
    seen = set()
    for _ in range(1500):
        ev = random_history(rng, rng.randint(0, 8), n_clients=rng.randint(1, 4))
        w, _ = orc.check_wgl(ev)
        b, _ = orc.check_brute(ev)
        assert w == b, ev
        seen.add(w)
    assert seen == {"Ok", "Illegal"}


def test_u64_regimes_wgl_brute_reduced_agree():
    """The u64 edges of s2Model.Step (main.go:279 wrap, main_test.go:313-343
    truncation) on concurrent histories: num_records independent of the hash
    count, tails across 2^32 and past 2^64, zero-record appends with hashes,
    match_seq_num = tail +- 2^32. Brute force = the WGL restatement = the
    reduced search with every reduction ablation; every code regime of the
    checker (tests/helpers.py u64_regime) gets both verdicts."""
    import collections

    from helpers import U64_REGIMES, random_history_u64, u64_regime
    rng = random.Random(5)
    seen = collections.Counter()
    for i in range(1200):
        ev = random_history_u64(rng, rng.randint(1, 9), n_clients=rng.randint(1, 4), regime=U64_REGIMES[i % 4])
        w, _ = orc.check_wgl(ev)
        assert orc.check_brute(ev)[0] == w, ev
        for off in (0, 1, 2, 4, 8):
            assert orc.check_reduced(ev, reductions_off=off)[0] == w, (off, ev)
        seen[(u64_regime(ev).split("+")[0], w)] += 1
        seen[("zh", w)] += "+zh" in u64_regime(ev)
    for r in ("tail32", "nowrap", "wrap", "zh"):
        assert seen[(r, "Ok")] >= 20 and seen[(r, "Illegal")] >= 20, seen


def test_reduced_search_on_u64_hard_variants():
    """H174's u64-regime variants (helpers.hard_variant) on the CPU reduced
    search against the committed H174 fixtures: a prepended 2^32-record append
    shifts the search by one round, exact match_seq_nums leave it unchanged, a
    prepended zero-record append with a hash gives the P2-off search, and a
    match_seq_num 2^32 above the true tail is Illegal."""
    import s2_verification_amd as s2
    from helpers import config_digest, golden, hard_variant

    from s2_verification_amd import workloads as W
    g = golden("hard_round_counts.json")["H174"]
    assert config_digest("H174") == g["digest"]
    ev = W.config_history("H174").events()
    want = {"above32": ("Ok", [1] + g["0"]["counts"]), "msn_exact": ("Ok", g["0"]["counts"]),
            "zero_hash": ("Ok", g["2"]["counts"])}
    for v in ("above32", "msn_exact", "zero_hash", "stale_msn"):
        hv = s2.History.from_events(hard_variant(ev, v))
        assert hv.info()["n_chains"] == 174
        r, st = orc.check_reduced(orc.from_s2lc_numpy(hv.events_numpy(), owner=hv), round_counts=True)
        if v == "stale_msn":
            assert r == "Illegal" and st["rounds"] < g["0"]["rounds"], (r, st["rounds"])
        else:
            assert (r, st["round_counts"]) == want[v], v


def test_unmatched_events_are_illegal():
    """A call without a return (or a return before its call) never leaves checkSingle's list."""
    call = {"kind": "call", "op_id": 1, "input_type": 1}
    ret = {"kind": "return", "op_id": 1, "failure": False, "definite_failure": False, "tail": 0,
           "stream_hash": 0}
    assert orc.check_wgl([call])[0] == "Illegal"
    assert orc.check_wgl([ret])[0] == "Illegal"
    assert orc.check_wgl([ret, call])[0] == "Illegal"
    assert orc.check_wgl([call, ret])[0] == "Ok"
    assert orc.check_wgl([])[0] == "Ok"


def test_model_panics_are_reported():
    """nil NumRecords on an append / nil Tail on a success: the Go model would panic."""
    call = {"kind": "call", "op_id": 1, "input_type": 0, "num_records": None, "record_hashes": []}
    ret = {"kind": "return", "op_id": 1, "failure": False, "definite_failure": False, "tail": 0}
    assert orc.check_wgl([call, ret])[0] == "Panic"


def test_call_left_last_in_the_list_panics_instead_of_crashing():
    """Two calls linked to one return can leave a call last in checkSingle's
    list; porcupine's lift then dereferences the call's nil next node. The
    restatement reports that panic (it used to dereference NULL itself)."""
    A = lambda i: {"kind": "call", "op_id": i, "input_type": 0, "num_records": 1, "record_hashes": [5 + i]}
    R = lambda i: {"kind": "return", "op_id": i, "failure": True, "definite_failure": False}
    v, st = orc.check_wgl([A(2), A(1), A(1), R(1), R(2)], compute_partial=True, timeout=5.0)
    assert v == "Panic" and st["cache_inserts"] == 3


def test_reduced_search_matches_wgl():
    """The CPU reduced search (cross-check oracle for C5) agrees with the WGL
    restatement on random histories and on simulator histories."""
    import s2_verification_amd as s2
    rng = random.Random(99)
    for _ in range(1500):
        ev = random_history(rng, rng.randint(0, 9), n_clients=rng.randint(1, 4))
        assert orc.check_reduced(ev)[0] == orc.check_wgl(ev)[0], ev
    for wf in (0, 1, 2):
        for seed in range(25):
            h = s2.simulate_history(workflow=wf, num_clients=4 + seed % 4, ops_per_client=60, seed=seed,
                                    violation=seed % 5, p_indefinite=0.03)
            ea = orc.from_s2lc_numpy(h.events_numpy())
            assert orc.check_reduced(ea)[0] == orc.check_wgl(ea)[0]


def test_reduced_search_ablations_agree_with_wgl():
    """oracle/reduced.c with each verdict-exact reduction switched off (the
    product's RED_* bits) gives porcupine's verdict (WGL restatement) on the
    bench workload and on random small histories, and its per-round counts
    account for every configuration it inserted."""
    import random

    from helpers import random_history
    from s2_verification_amd import workloads as W
    hs = [orc.from_s2lc_numpy(h.events_numpy()) for h in W.c4_histories(120, first_seed=4000)]
    rng = random.Random(3)
    hs += [random_history(rng, rng.randint(1, 9), n_clients=rng.randint(1, 4)) for _ in range(300)]
    for ev in hs:
        w, _ = orc.check_wgl(ev)
        for off in range(16):
            v, st = orc.check_reduced(ev, reductions_off=off, round_counts=True)
            assert v == w, (off, v, w)
            assert len(st["round_counts"]) == st["rounds"]
            if v == "Illegal":  # every round completed: the counts are all the configurations (+ round 0)
                assert sum(st["round_counts"]) == st["configs"] + (1 if st["rounds"] else 0)


def test_reduced_p2_only_prunes():
    """P2 (a minimal read at the current tail with another hash is dead) only
    removes configurations: per-round counts with it on never exceed those
    with it off, and the rounds are the same (hard fixtures, committed)."""
    from helpers import golden
    g = golden("hard_round_counts.json")
    for name in ("H174", "H212", "C5bad"):
        on, off = g[name]["0"], g[name]["2"]
        assert on["verdict"] == off["verdict"]
        if on["verdict"] == "Ok":
            assert on["rounds"] == off["rounds"]
        assert all(a <= b for a, b in zip(on["counts"], off["counts"]))


def test_reduced_search_reproduces_the_complete_ablation_fixtures():
    """The committed whole-search ablations on > 128 chains (A144 / A160,
    make_round_counts.py) are what oracle/reduced.c gives now, for those
    that finish in about a second here; every ablation is a superset of the
    all-on search round by round (a reduction only removes configurations)."""
    from helpers import config_digest, golden

    from s2_verification_amd import workloads as W
    g = golden("hard_round_counts.json")
    for name, offs in (("A144", (0, 2, 8)), ("A160", (0, 2))):
        assert config_digest(name) == g[name]["digest"]
        h = W.config_history(name)
        assert h.info()["n_chains"] > 128
        ea = orc.from_s2lc_numpy(h.events_numpy(), owner=h)
        for off in offs:
            v, st = orc.check_reduced(ea, reductions_off=off, round_counts=True)
            want = g[name][str(off)]
            assert (v, st["rounds"], st["round_counts"]) == (want["verdict"], want["rounds"], want["counts"])
    for name in ("A144", "A160"):
        on = g[name]["0"]["counts"]
        for off in ("1", "2", "8"):
            if off in g[name]:
                assert g[name][off]["verdict"] == "Ok" and g[name][off]["rounds"] == g[name]["0"]["rounds"]
                assert all(a <= b for a, b in zip(on, g[name][off]["counts"]))


def test_from_s2lc_numpy_owns_its_hashes():
    """Without the owning history, the oracle's event array copies the record
    hashes: checking it after the history is gone gives the same verdict and
    search as with the history alive (a use-after-free before the copy)."""
    import gc

    from s2_verification_amd import workloads as W
    h = W.c4_histories(1, first_seed=4007)[0]
    with_owner = orc.from_s2lc_numpy(h.events_numpy(), owner=h)
    v1, st1 = orc.check_reduced(with_owner, round_counts=True)
    ea = orc.from_s2lc_numpy(h.events_numpy())
    del h, with_owner
    gc.collect()
    junk = [bytearray(1 << 16) for _ in range(64)]  # reuse the freed memory
    v2, st2 = orc.check_reduced(ea, round_counts=True)
    assert (v1, st1["round_counts"]) == (v2, st2["round_counts"])
    del junk
