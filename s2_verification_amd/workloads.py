"""The five BASELINE.json configurations as deterministic-simulator parameters.

SURVEY.md §8(d): C1 regular 5x100 (seed 1), C2 match-seq-num 10x200 (seed 2),
C3 fencing 16x500 (seed 3), C4 10k histories of 5-8 clients x 100 ops (seeds
0..9999, clients = 5 + seed mod 4, workflow = seed mod 3, every 10th seed with
an injected violation), C5 32x1000 (seed 5, client-id cap lifted, 3% indefinite
appends) and its non-linearizable variant.
"""
from . import (VIOL_DEFINITE_APPLIED, VIOL_NONE, VIOL_READ_HASH, VIOL_STALE_MSN, VIOL_TAIL, WF_FENCING,
               WF_MATCH_SEQ_NUM, WF_REGULAR, sim_params, simulate_history, simulate_jsonl)

BASE = dict(p_indefinite=0.01, p_definite=0.02, p_read_failure=0.01, p_check_tail_failure=0.01)

CONFIGS = {
    "C1": dict(workflow=WF_REGULAR, num_clients=5, ops_per_client=100, seed=1, **BASE),
    "C2": dict(workflow=WF_MATCH_SEQ_NUM, num_clients=10, ops_per_client=200, seed=2, **BASE),
    "C3": dict(workflow=WF_FENCING, num_clients=16, ops_per_client=500, seed=3, **BASE),
    # single hard history: the client-id cap is lifted (max_client_ids), so a
    # client that hits an indefinite failure rotates to a new id and keeps
    # going (DST-harness style) instead of stopping at id 20 (history.rs:153-169);
    # with 3% indefinite appends this leaves ~290 pending appends whose
    # outcome only later reads resolve: K = 319 chains, ~1.6 M unique
    # configurations, ~175 M children (the CPU reduced search needs minutes,
    # porcupine's DFS does not finish).
    "C5": dict(workflow=WF_REGULAR, num_clients=32, ops_per_client=1000, seed=5, max_client_ids=1 << 20,
               **{**BASE, "p_indefinite": 0.03}),
    "C5bad": dict(workflow=WF_REGULAR, num_clients=32, ops_per_client=1000, seed=5, max_client_ids=1 << 20,
                  violation=VIOL_READ_HASH, **{**BASE, "p_indefinite": 0.03}),
    # a single hard history whose WIDE rounds dominate (the shape the
    # distributed search partitions): 24 clients x 300 ops with 10% indefinite
    # appends, K = 243 chains; 30 of its 2,231 rounds hold 1.03 M of its 1.11 M
    # unique configurations (frontier up to 273 k); CPU reduced search ~2 min
    "C5wide": dict(workflow=WF_REGULAR, num_clients=24, ops_per_client=300, seed=12, max_client_ids=1 << 20,
                   **{**BASE, "p_indefinite": 0.10}),
    # mid-size hard histories (level-search parity against the CPU reduced search)
    "H174": dict(workflow=WF_REGULAR, num_clients=32, ops_per_client=1000, seed=5, max_client_ids=1 << 20,
                 **{**BASE, "p_indefinite": 0.015}),
    "H212": dict(workflow=WF_REGULAR, num_clients=32, ops_per_client=1000, seed=6, max_client_ids=1 << 20,
                 **{**BASE, "p_indefinite": 0.02}),
    # 32 < K <= 128 (the workgroup-per-history engine, search_kernel): many
    # clients with the collector's client-id cap (ids start above 20, so a
    # client stops at its first indefinite failure); porcupine's DFS does not
    # finish on them, the CPU reduced search does in milliseconds
    "H48": dict(workflow=WF_REGULAR, num_clients=48, ops_per_client=200, seed=7, **{**BASE, "p_indefinite": 0.003}),
    "H48bad": dict(workflow=WF_REGULAR, num_clients=48, ops_per_client=200, seed=7, violation=VIOL_READ_HASH,
                   **{**BASE, "p_indefinite": 0.003}),
    "H96": dict(workflow=WF_REGULAR, num_clients=96, ops_per_client=80, seed=3, **BASE),
    "H100": dict(workflow=WF_REGULAR, num_clients=100, ops_per_client=60, seed=9, **{**BASE, "p_indefinite": 0.003}),
    "H120m": dict(workflow=WF_MATCH_SEQ_NUM, num_clients=120, ops_per_client=50, seed=9,
                  **{**BASE, "p_indefinite": 0.003}),
    # > 128 chains with every reduction ablation finishing on the CPU (whole-
    # search ablation fixtures, tests/golden/make_round_counts.py): many
    # clients with the client-id cap, few ops each. A144: P1 off 4.9 M unique
    # configurations, deferral off 36 k; A160: deferral off 4.2 M (P1 off
    # does not finish)
    "A144": dict(workflow=WF_REGULAR, num_clients=144, ops_per_client=16, seed=21, **{**BASE, "p_indefinite": 0.02}),
    "A160": dict(workflow=WF_REGULAR, num_clients=160, ops_per_client=20, seed=13, **{**BASE, "p_indefinite": 0.03}),
    # the round-1 C5 (client-id cap 20: clients stop at their first indefinite failure)
    "C5capped": dict(workflow=WF_REGULAR, num_clients=32, ops_per_client=1000, seed=5,
                     **{**BASE, "p_indefinite": 0.002}),
}

_C4_VIOLS = [VIOL_READ_HASH, VIOL_TAIL, VIOL_DEFINITE_APPLIED, VIOL_STALE_MSN]


def c4_params(seed: int) -> dict:
    """One history of the C4 batch (DST seed `seed`)."""
    wf = (WF_REGULAR, WF_MATCH_SEQ_NUM, WF_FENCING)[seed % 3]
    viol = _C4_VIOLS[(seed // 10) % 4] if seed % 10 == 7 else VIOL_NONE
    return dict(workflow=wf, num_clients=5 + seed % 4, ops_per_client=100, seed=seed, violation=viol, **BASE)


def config_meta(name: str) -> dict:
    """What a config name promises against what the simulator is asked for:
    the planned op count (clients x ops per client) and the client-id cap
    (the collector's MAX_CLIENT_IDS = 20, history.rs:33, unless lifted). Under
    the cap a client stops at its first indefinite failure once its ids run
    out, so a history can hold fewer ops than planned (C3: 4,325 of 8,000)."""
    c = CONFIGS[name]
    p = sim_params(**c)
    return {"n_ops_planned": c["num_clients"] * c["ops_per_client"], "client_id_cap": int(p.max_client_ids),
            "client_id_cap_lifted": int(p.max_client_ids) != COLLECTOR_MAX_CLIENT_IDS}


COLLECTOR_MAX_CLIENT_IDS = 20  # collect-history's MAX_CLIENT_IDS (history.rs:33)


def config_history(name: str):
    return simulate_history(**CONFIGS[name])


def config_jsonl(name: str) -> bytes:
    return simulate_jsonl(**CONFIGS[name])


def c4_histories(n: int = 10000, first_seed: int = 0):
    return [simulate_history(**c4_params(s)) for s in range(first_seed, first_seed + n)]
