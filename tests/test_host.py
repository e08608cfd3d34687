"""CPU: the C-ABI library loads and exports every declared symbol; host logic
(model step, chain decomposition, replay, simulator) against the oracle."""
import os
import random
import re

import oracle as orc
import s2_verification_amd as s2
from helpers import golden, random_history, to_s2_events

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "s2lincheck.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(s2lc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = s2.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    for name in syms:
        assert hasattr(L, name), name
    assert {n for n, _, _ in s2.SIGNATURES} == set(syms)


def test_chain_hash_matches_golden():
    g = golden("chain_hash_vectors.json")
    for h, r, want in g["pairs"]:
        assert s2.chain_hash(h, r) == want
    for h, rs, want in g["folds"]:
        assert s2.fold_record_hashes(h, rs) == want


def test_history_info_and_chains():
    for wf in (0, 1, 2):
        h = s2.simulate_history(workflow=wf, num_clients=6, ops_per_client=80, seed=3)
        info = h.info()
        assert info["n_events"] == 2 * info["n_ops"]
        assert 1 <= info["n_chains"] <= 6 + 20  # clients + rotated ids
        assert info["structural"] == 0


def test_step_cpu_matches_oracle_model():
    """s2lc_step_cpu == the oracle's s2Model.Step on single-op histories from many states."""
    rng = random.Random(5)
    for _ in range(300):
        ev = random_history(rng, 1, n_clients=1, p_perturb=0.5)
        h = s2.History.from_events(to_s2_events(ev))
        got0 = h.step((0, 0, 0), 0)  # from Init; the oracle's verdict on a 1-op history is the same test
        w, _ = orc.check_wgl(ev)
        assert (len(got0) > 0) == (w == "Ok"), (ev, got0, w)


def test_replay_accepts_valid_and_rejects_invalid_orders():
    for c in golden("reference_cases.json")["cases"]:
        h = s2.History.from_events(to_s2_events(c["events"]))
        n = h.info()["n_ops"]
        assert h.replay(list(range(n))) == (c["expected"] == "Ok"), c["name"]
    h = s2.History.from_events(to_s2_events(golden("reference_cases.json")["cases"][1]["events"]))
    assert not h.replay([1, 0, 2])      # read before the append it observes
    assert not h.replay([0, 1])         # not a permutation
    assert not h.replay([0, 0, 1])


def test_unmatched_history_structural_flag():
    ev = [{"kind": "call", "op_id": 1, "input_type": 1}]
    h = s2.History.from_events(to_s2_events(ev))
    assert h.info()["structural"] == 1


def test_duplicate_op_ids_take_the_literal_engine():
    """Repeated op ids (porcupine accepts them): the history builds without
    chains; its ops are the call events, each linked to the nearest later
    return with its id (makeLinkedEntries)."""
    ev = [{"kind": "call", "op_id": 1, "input_type": 1},
          {"kind": "return", "op_id": 1, "failure": True, "definite_failure": True},
          {"kind": "call", "op_id": 1, "input_type": 1},
          {"kind": "return", "op_id": 1, "failure": True, "definite_failure": True}]
    h = s2.History.from_events(to_s2_events(ev))
    info = h.info()
    assert info["n_ops"] == 2 and info["n_chains"] == 0 and info["structural"] == 0
    # porcupine's quirk with a repeated id: the second op sets the bit the
    # first already set, so its cache entry equals the first's and the search
    # prunes it: Illegal, although the ops are sequential and both legal
    assert orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy()))[0] == "Illegal"


def test_simulated_histories_linearizable_by_oracle():
    """Clean simulator output is linearizable by construction; violations make it Illegal."""
    for wf in (0, 1, 2):
        for seed in range(4):
            h = s2.simulate_history(workflow=wf, num_clients=5, ops_per_client=60, seed=seed, p_indefinite=0.03)
            assert orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy()))[0] == "Ok"
    bad = 0
    for v in (s2.VIOL_READ_HASH, s2.VIOL_TAIL, s2.VIOL_DEFINITE_APPLIED, s2.VIOL_STALE_MSN):
        for seed in range(3):
            h = s2.simulate_history(workflow=1, num_clients=5, ops_per_client=60, seed=seed, violation=v)
            bad += orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy()))[0] == "Illegal"
    assert bad >= 10


def test_simulator_deterministic():
    a = s2.simulate_jsonl(workflow=2, num_clients=5, ops_per_client=40, seed=9)
    b = s2.simulate_jsonl(workflow=2, num_clients=5, ops_per_client=40, seed=9)
    c = s2.simulate_jsonl(workflow=2, num_clients=5, ops_per_client=40, seed=10)
    assert a == b and a != c


def test_fence_token_hash_is_xxh3():
    """Fence-command record hash = xxh3_64(token bytes) (history.rs:202)."""
    import json

    import xxhash
    data = s2.simulate_jsonl(workflow=2, num_clients=3, ops_per_client=5, seed=1)
    n = 0
    for line in data.splitlines():
        rec = json.loads(line)
        st = rec["event"].get("Start")
        if isinstance(st, dict) and st["Append"]["set_fencing_token"]:
            tok = st["Append"]["set_fencing_token"]
            assert st["Append"]["record_hashes"] == [xxhash.xxh3_64_intdigest(tok.encode())]
            n += 1
    assert n >= 3


def test_bench_watchdog_exits_nonzero_with_the_stalled_leg():
    """bench.py's multi-GPU watchdog, on the CPU: a leg
    that outlives S2LC_BENCH_WATCHDOG makes rank 0 print the line it has so
    far with `stalled_leg`, and the process exit with WATCHDOG_EXIT (non-zero:
    a stalled collective never reads as success); a disarmed timer never
    fires."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "line = {'metric': 'm', 'value': 1.0}; wd = bench._Watchdog(0, line); "
            "wd.arm('quick'); wd.disarm(); time.sleep(0.3); "
            "line['quick'] = {'ok': True}; wd.arm('stuck'); time.sleep(30)" % root)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, S2LC_BENCH_WATCHDOG="0.2"))
    import bench  # noqa: E402  (the exit code it promises)
    assert p.returncode == bench.WATCHDOG_EXIT != 0, (p.returncode, p.stderr[-2000:])
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["stalled_leg"] == "stuck" and d["quick"] == {"ok": True} and "watchdog" in d, d
