"""LinearizationInfo parity (porcupine.CheckEventsVerbose's second result,
main.go:606, rendered by Visualize at main.go:627): for every op, the length
of the longest partial linearization containing it equals what porcupine's
DFS records (oracle/oracle.c computePartial: longest[] on every backtrack).

GPU: s2lc_check_partials (the unreduced level search recording per-op
maxima, every distinct partial rebuilt and certified) against the oracle on
small Illegal histories and C4 Illegal histories; CPU: the oracle's own
lengths on linearizable histories (every op: the whole history)."""
import random

import pytest

import oracle as orc
import s2_verification_amd as s2
from helpers import from_s2_events, random_history, to_s2_events


def _dense_ids(events):
    """op ids in porcupine renumber order (first appearance)."""
    seen, out = set(), []
    for e in events:
        if e["op_id"] not in seen:
            seen.add(e["op_id"])
            out.append(e["op_id"])
    return out


def test_oracle_longest_on_ok_is_everything():
    rng = random.Random(3)
    n_ok = 0
    for _ in range(200):
        ev = random_history(rng, rng.randint(1, 8), 3, p_perturb=0.0)
        v, lens = orc.check_wgl_longest(ev)
        if v == "Ok":
            n_ok += 1
            n = len(_dense_ids(ev))
            assert list(lens[:n]) == [n] * n
    assert n_ok > 100


def _compare(checker, ev):
    w, lens = orc.check_wgl_longest(ev, timeout=30.0)
    if w == "Unknown":
        return None
    h = s2.History.from_events(to_s2_events(ev))
    info = checker.partials(h)
    assert info.verdict == w, (info.verdict, w)
    if w != "Illegal":
        return w
    assert info.exact
    for d, op in enumerate(_dense_ids(ev)):
        k = info.largest[op]
        got = 0 if k is None else len(info.partial_linearizations[k])
        assert got == lens[d], (op, got, int(lens[d]))
        if k is not None:
            assert op in info.partial_linearizations[k]
    return w


@pytest.mark.gpu
def test_partials_match_porcupine_longest_small(checker):
    rng = random.Random(17)
    n_ill = 0
    for _ in range(300):
        ev = random_history(rng, rng.randint(2, 9), rng.randint(1, 4), p_perturb=0.3)
        n_ill += _compare(checker, ev) == "Illegal"
    assert n_ill > 50


@pytest.mark.gpu
def test_partials_match_porcupine_longest_c4_illegal(checker):
    from s2_verification_amd import workloads as W
    n_ill = 0
    for sd in range(7, 400, 10):  # every C4 seed with an injected violation
        h = s2.simulate_history(**W.c4_params(sd))
        if _compare(checker, from_s2_events(h.events())) == "Illegal":
            n_ill += 1
    assert n_ill >= 30


@pytest.mark.gpu
def test_partials_on_ok_are_the_witness(checker):
    from s2_verification_amd import workloads as W
    h = W.config_history("C1")
    info = checker.partials(h)
    r = checker.check(h)
    assert info.verdict == s2.Ok and len(info.partial_linearizations) == 1
    assert info.partial_linearizations[0] == r.witness
    assert set(info.largest.values()) == {0}
