"""The full C4 batch (BASELINE.json configs[3]: 10,000 DST-seed histories, 5-8
clients x 100 ops, three workflows, every 10th seed with an injected violation)
on the GPU: exactly the batch bench.py times, checked history by history
against the CPU results committed in tests/golden/c4_verdicts.json
(tests/golden/make_c4_golden.py):

  * verdict = porcupine's WGL restated (oracle/oracle.c, computePartial on);
  * every Ok carries a witness certified by the library's CPU replay;
  * rounds and the per-round unique-configuration counts = the CPU reduced
    search (oracle/reduced.c), and for Illegal histories (whole search
    space) the total unique configurations too (the GPU counts round 0's
    initial configuration, oracle/reduced.c does not).

The simulator output is pinned by a digest of the batch's collector JSONL.
"""
import hashlib

import numpy as np
import pytest

import s2_verification_amd as s2
from helpers import golden

pytestmark = pytest.mark.gpu

V = {"O": s2.Ok, "I": s2.Illegal, "U": s2.Unknown}


@pytest.fixture(scope="module")
def c4():
    from s2_verification_amd import workloads as W
    ref = golden("c4_verdicts.json")
    n = ref["n"]
    hsh = hashlib.sha256()
    for sd in range(n):
        hsh.update(s2.simulate_jsonl(**W.c4_params(sd)))
    assert hsh.hexdigest()[:32] == ref["simulator_jsonl_sha256"], "simulator output changed: regenerate the fixture"
    return ref, W.c4_histories(n)


def test_c4_full_batch_verdicts_and_certified_witnesses(c4):
    """bench.py's checker (witnesses on, default engines) over the whole batch."""
    ref, hs = c4
    b = s2.Checker().batch(hs)
    b.run()
    st = b.stats()
    flat = b.results_flat(with_witness=True)  # raises on any witness that fails CPU replay
    want = np.array([s2.S2LC_OK if r[0] == "O" else s2.S2LC_ILLEGAL for r in ref["rows"]], np.int32)
    got = flat["verdict"]
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, ("verdict mismatches at seeds", bad[:10].tolist())
    offs = flat["witness_offs"].astype(np.int64)
    wl = np.diff(offs)
    n_ops = np.array([h.info()["n_ops"] for h in hs], np.int64)
    ok = want == s2.S2LC_OK
    assert (wl[ok] == n_ops[ok]).all(), "an Ok without a full certified witness"
    assert (wl[~ok] == 0).all()
    # every op exactly once in each witness
    for i in np.nonzero(ok)[0][::97]:
        w = flat["witness_ids"][offs[i]:offs[i + 1]]
        assert len(np.unique(w)) == n_ops[i]
    assert int(ok.sum()) == 9001 and int((~ok).sum()) == 999
    assert st["pack16_histories"] + st["pack8_histories"] >= 9900, st  # the bench's dominant kernel ran them


def test_c4_full_batch_round_counts(c4):
    """Per history: rounds, per-round unique-configuration counts (digest) and,
    for Illegal, total unique configurations = the CPU reduced search."""
    ref, hs = c4
    b = s2.Checker(round_counts=True).batch(hs)
    res = b.check(with_witness=False)
    mism = []
    for i, (r, row) in enumerate(zip(res, ref["rows"])):
        wv, _, rv, rounds, configs, dig = row
        counts = b.round_counts(i)
        d = hashlib.sha256(np.asarray(counts, dtype="<u4").tobytes()).hexdigest()[:16]
        if r.verdict != V[rv] or r.rounds != rounds or d != dig or (rv == "I" and r.configs_explored != configs + 1):
            mism.append((i, r.verdict, rv, r.rounds, rounds, r.configs_explored, configs))
    assert not mism, (len(mism), mism[:5])
