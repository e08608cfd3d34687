"""Test helpers: golden fixtures, event conversion, random small histories.

Random histories come from a sequential ground-truth execution with random
real-time intervals around each linearization point, then optional output
perturbations, so both Ok and Illegal verdicts occur. Their verdict is
decided by the oracle (WGL restatement, cross-checked by brute force).
"""
import json
import os
import random

import s2_verification_amd as s2

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def to_s2_events(events):
    """oracle dict events -> s2_verification_amd.Event list."""
    out = []
    for e in events:
        if e["kind"] == "call":
            v = s2.StreamInput(InputType=e["input_type"], SetFencingToken=e.get("set_fencing_token"),
                               BatchFencingToken=e.get("fencing_token"), MatchSeqNum=e.get("match_seq_num"),
                               NumRecords=e.get("num_records"), RecordHashes=list(e.get("record_hashes") or []))
            out.append(s2.Event(s2.CallEvent, v, e["op_id"], e.get("client_id", 0)))
        else:
            v = s2.StreamOutput(Failure=e["failure"], DefiniteFailure=e["definite_failure"], Tail=e.get("tail"),
                                StreamHash=e.get("stream_hash"))
            out.append(s2.Event(s2.ReturnEvent, v, e["op_id"], e.get("client_id", 0)))
    return out


def from_s2_events(events):
    """s2_verification_amd.Event list -> oracle dict events."""
    out = []
    for e in events:
        v = e.Value
        if e.Kind == s2.CallEvent:
            out.append({"kind": "call", "op_id": e.Id, "client_id": e.ClientId, "input_type": v.InputType,
                        "num_records": v.NumRecords, "match_seq_num": v.MatchSeqNum,
                        "set_fencing_token": v.SetFencingToken, "fencing_token": v.BatchFencingToken,
                        "record_hashes": list(v.RecordHashes)})
        else:
            out.append({"kind": "return", "op_id": e.Id, "client_id": e.ClientId, "failure": v.Failure,
                        "definite_failure": v.DefiniteFailure, "tail": v.Tail, "stream_hash": v.StreamHash})
    return out


def _fold(h, rs):
    for r in rs:
        h = s2.chain_hash(h, r)
    return h


def random_history(rng: random.Random, n_ops: int, n_clients: int = 3, p_perturb: float = 0.15,
                   tokens=("aaaaaa", "bbbbbb")):
    """A random small history over n_clients (events as oracle dicts)."""
    tail, h, tok = 0, 0, None
    ops = []
    t = 0.0
    for i in range(n_ops):
        kind = rng.choice(["append", "append", "read", "check_tail"])
        op = {"op_id": i, "client_id": rng.randrange(n_clients)}
        lin = t = t + rng.random()
        op["call"] = lin - rng.random() * 3.0
        op["ret"] = lin + rng.random() * 3.0
        if kind == "append":
            nrec = rng.randint(0, 3)
            hs = [rng.getrandbits(64) for _ in range(nrec)]
            set_tok = rng.choice(tokens) if rng.random() < 0.15 else None
            batch_tok = rng.choice(tokens) if rng.random() < 0.15 else None
            msn = (tail if rng.random() < 0.7 else tail + rng.randint(1, 3)) if rng.random() < 0.3 else None
            guards = (batch_tok is None or batch_tok == tok) and (msn is None or msn == tail)
            r = rng.random()
            call = {"input_type": 0, "num_records": nrec, "record_hashes": hs, "set_fencing_token": set_tok,
                    "fencing_token": batch_tok, "match_seq_num": msn}
            if r < 0.2:
                applied = guards and rng.random() < 0.5
                out = {"failure": True, "definite_failure": False, "tail": None, "stream_hash": None}
            elif r < 0.3 or not guards:
                applied = False
                out = {"failure": True, "definite_failure": True, "tail": None, "stream_hash": None}
            else:
                applied = True
                out = None
            if applied:
                tail += nrec
                h = _fold(h, hs)
                if set_tok is not None:
                    tok = set_tok
            if out is None:
                out = {"failure": False, "definite_failure": False, "tail": tail, "stream_hash": None}
        elif kind == "read":
            call = {"input_type": 1}
            if rng.random() < 0.1:
                out = {"failure": True, "definite_failure": True, "tail": None, "stream_hash": None}
            else:
                out = {"failure": False, "definite_failure": False, "tail": tail, "stream_hash": h}
        else:
            call = {"input_type": 2}
            if rng.random() < 0.1:
                out = {"failure": True, "definite_failure": True, "tail": None, "stream_hash": None}
            else:
                out = {"failure": False, "definite_failure": False, "tail": tail, "stream_hash": None}
        if rng.random() < p_perturb:
            if out["tail"] is not None and rng.random() < 0.5:
                out["tail"] += rng.choice([-1, 1]) if out["tail"] > 0 else 1
            elif out["stream_hash"] is not None:
                out["stream_hash"] ^= 1 << rng.randrange(64)
            elif out["failure"] and kind == "append":
                out["definite_failure"] = not out["definite_failure"]
        op.update(call_fields=call, out=out)
        ops.append(op)
    evs = []
    for op in ops:
        evs.append((op["call"], 0, {"kind": "call", "op_id": op["op_id"], "client_id": op["client_id"],
                                    **op["call_fields"]}))
        evs.append((op["ret"], 1, {"kind": "return", "op_id": op["op_id"], "client_id": op["client_id"],
                                   **op["out"]}))
    evs.sort(key=lambda x: (x[0], x[1]))
    return [e for _, _, e in evs]


M64 = (1 << 64) - 1
U64_REGIMES = ("tail32_edge", "above32", "wrap", "zero_hashes")


def random_history_u64(rng: random.Random, n_ops: int, n_clients: int = 3, regime: str = "tail32_edge",
                       p_perturb: float = 0.15, tokens=("aaaaaa", "bbbbbb")):
    """A random small history over the u64 edges of s2Model.Step
    (main.go:264-335), the bug class main_test.go:313-343 pins, and over the
    16-bit fields of the packed kernels' 32-byte records ("small_edge": the
    first append leaves the tail at 65,520 .. 65,532, later appends carry
    65,535 .. 65,537 records now and then, match_seq_num = tail +- 2^16 and
    0xFFFD .. 0x10000, success tails perturbed by +-2^16):

      - num_records drawn independently of the record-hash count (expressible
        only through the event API, main_test.go:322);
      - tails near 2^32 - 4 .. 2^32 + 5 ("tail32_edge": the first append leaves
        the tail a few records below 2^32 - 3), beyond 2^32 ("above32"), and
        sums of num_records past 2^63 whose tails wrap mod 2^64 ("wrap",
        main.go:279);
      - zero-record appends that carry record hashes ("zero_hashes");
      - match_seq_num = tail + 2^32 or tail - 2^32 (equal to the true tail in
        its low 32 bits), beside the true tail and tail +- 1;
      - success tails perturbed by +-2^32 as well as +-1.

    Ground truth is a sequential execution with random real-time intervals
    around each linearization point (as random_history), events as oracle
    dicts; verdicts come from the oracle."""
    tail, h, tok = 0, 0, None
    ops = []
    t = 0.0
    first_append = True
    for i in range(n_ops):
        kind = rng.choice(["append", "append", "append", "read", "check_tail"])
        op = {"op_id": i, "client_id": rng.randrange(n_clients)}
        lin = t = t + rng.random()
        op["call"] = lin - rng.random() * 3.0
        op["ret"] = lin + rng.random() * 3.0
        if kind == "append":
            nh = rng.randint(0, 3)
            nrec = rng.randint(0, 3)  # independent of nh
            if regime == "tail32_edge" and first_append:
                nrec = (1 << 32) - 4 - rng.randint(0, 10)
            elif regime == "above32" and rng.random() < 0.4:
                nrec = rng.choice([(1 << 32) + rng.randint(-3, 5), 1 << 33, (1 << 32) - rng.randint(1, 4)])
            elif regime == "wrap" and rng.random() < 0.45:
                nrec = rng.choice([(1 << 63) + rng.randint(0, 3), (1 << 64) - rng.randint(1, 5),
                                   (1 << 63) - rng.randint(0, 3)])
            elif regime == "zero_hashes" and rng.random() < 0.5:
                nrec, nh = 0, rng.randint(1, 2)
            elif regime == "small_edge" and first_append:
                nrec = 65532 - rng.randint(0, 12)
            elif regime == "small_edge" and rng.random() < 0.08:
                nrec = rng.choice([65535, 65536, 65537])
            elif nrec == 0 and regime != "zero_hashes" and rng.random() < 0.9:
                nh = 0  # (keep P2 on in most histories of the other regimes)
            first_append = False
            hs = [rng.getrandbits(64) for _ in range(nh)]
            set_tok = rng.choice(tokens) if rng.random() < 0.15 else None
            batch_tok = rng.choice(tokens) if rng.random() < 0.15 else None
            msn = None
            if rng.random() >= 0.4:
                pass
            elif regime == "small_edge":
                msn = rng.choice([tail, tail, tail + 65536, (tail - 65536) & M64, tail + 1, (tail - 1) & M64,
                                  0xFFFD, 0xFFFE, 0xFFFF, 0x10000])
            else:
                msn = rng.choice([tail, tail, (tail + (1 << 32)) & M64, (tail - (1 << 32)) & M64,
                                  (tail + 1) & M64, (tail - 1) & M64])
            guards = (batch_tok is None or batch_tok == tok) and (msn is None or msn == tail)
            r = rng.random()
            call = {"input_type": 0, "num_records": nrec, "record_hashes": hs, "set_fencing_token": set_tok,
                    "fencing_token": batch_tok, "match_seq_num": msn}
            if r < 0.2:
                applied = guards and rng.random() < 0.5
                out = {"failure": True, "definite_failure": False, "tail": None, "stream_hash": None}
            elif r < 0.3 or not guards:
                applied = False
                out = {"failure": True, "definite_failure": True, "tail": None, "stream_hash": None}
            else:
                applied = True
                out = None
            if applied:
                tail = (tail + nrec) & M64
                h = _fold(h, hs)
                if set_tok is not None:
                    tok = set_tok
            if out is None:
                out = {"failure": False, "definite_failure": False, "tail": tail, "stream_hash": None}
        elif kind == "read":
            call = {"input_type": 1}
            if rng.random() < 0.1:
                out = {"failure": True, "definite_failure": True, "tail": None, "stream_hash": None}
            else:
                out = {"failure": False, "definite_failure": False, "tail": tail, "stream_hash": h}
        else:
            call = {"input_type": 2}
            if rng.random() < 0.1:
                out = {"failure": True, "definite_failure": True, "tail": None, "stream_hash": None}
            else:
                out = {"failure": False, "definite_failure": False, "tail": tail, "stream_hash": None}
        if rng.random() < p_perturb:
            if out["tail"] is not None and rng.random() < 0.6:
                d = [-1, 1, 65536, -65536] if regime == "small_edge" else [-1, 1, 1 << 32, -(1 << 32)]
                out["tail"] = (out["tail"] + rng.choice(d)) & M64
            elif out["stream_hash"] is not None:
                out["stream_hash"] ^= 1 << rng.randrange(64)
            elif out["failure"] and kind == "append":
                out["definite_failure"] = not out["definite_failure"]
        op.update(call_fields=call, out=out)
        ops.append(op)
    evs = []
    for op in ops:
        evs.append((op["call"], 0, {"kind": "call", "op_id": op["op_id"], "client_id": op["client_id"],
                                    **op["call_fields"]}))
        evs.append((op["ret"], 1, {"kind": "return", "op_id": op["op_id"], "client_id": op["client_id"],
                                   **op["out"]}))
    evs.sort(key=lambda x: (x[0], x[1]))
    return [e for _, _, e in evs]


def u64_regime(events) -> str:
    """Which of the checker's code regimes a history falls in (the product's
    history flags, csrc/history.cpp finalize, restated): 'tail32' (every
    reachable tail below 2^32 - 3), 'nowrap' (sum of num_records <= 2^63,
    64-bit tails), 'wrap' (P1 / P2 off); '+zh' when a zero-record append
    carries hashes (P2 off)."""
    total, nowrap, zh = 0, True, False
    for e in events:
        if e["kind"] != "call" or e["input_type"] != 0:
            continue
        n = e["num_records"]
        if n > (1 << 63) - total:
            nowrap = False
        else:
            total += n
        if n == 0 and e.get("record_hashes"):
            zh = True
    r = ("tail32" if total <= 0xFFFFFFFC else "nowrap") if nowrap else "wrap"
    return r + ("+zh" if zh else "")


def _success_append_ops(evs):
    """{op id: (call event, return event)} of the successful appends."""
    calls = {e.Id: e for e in evs if e.Kind == s2.CallEvent}
    out = {}
    for e in evs:
        if e.Kind == s2.ReturnEvent and not e.Value.Failure and calls[e.Id].Value.InputType == 0:
            out[e.Id] = (calls[e.Id], e)
    return out


def hard_variant(events, variant: str):
    """u64-regime variants of a hard single history (s2_verification_amd.Event
    list, e.g. H174's), built on the event API (num_records independent of the
    hash count, main_test.go:322):

      above32    an append of num_records = 2^32 with no record hashes,
                 returned before every other call, and every success tail
                 shifted by 2^32: the same search one round later (round
                 counts [1] + the original's), with 64-bit tails
                 (not H_TAIL32: the grid rounds' 64-bit P1, no solo rounds)
      msn_exact  every successful append guarded by match_seq_num = its true
                 pre-tail (out tail - num_records): the same search (a
                 success already pins the pre-tail, main.go:301-318)
      stale_msn  one successful append mid-history guarded by its pre-tail +
                 2^32 (equal in the low 32 bits, main_test.go:325-335):
                 Illegal
      zero_hash  a definite-failed append of 0 records carrying a hash,
                 returned before every other call: P2 off (the original's
                 P2-off search, same rounds)
    """
    evs = [s2.Event(e.Kind, type(e.Value)(**vars(e.Value)), e.Id, e.ClientId) for e in events]
    new_id = max(e.Id for e in evs) + 1
    if variant in ("above32", "zero_hash"):
        for e in evs:
            if variant == "above32" and e.Kind == s2.ReturnEvent and not e.Value.Failure:
                e.Value.Tail += 1 << 32
        if variant == "above32":
            pre = [s2.Event(s2.CallEvent, s2.StreamInput(InputType=0, NumRecords=1 << 32, RecordHashes=[]), new_id),
                   s2.Event(s2.ReturnEvent, s2.StreamOutput(Tail=1 << 32), new_id)]
        else:
            pre = [s2.Event(s2.CallEvent, s2.StreamInput(InputType=0, NumRecords=0, RecordHashes=[0x5eed]), new_id),
                   s2.Event(s2.ReturnEvent, s2.StreamOutput(Failure=True, DefiniteFailure=True), new_id)]
        return pre + evs
    ops = _success_append_ops(evs)
    if variant == "msn_exact":
        for c, r in ops.values():
            c.Value.MatchSeqNum = r.Value.Tail - c.Value.NumRecords
    elif variant == "stale_msn":
        ids = sorted(ops)
        c, r = ops[ids[len(ids) // 2]]
        c.Value.MatchSeqNum = r.Value.Tail - c.Value.NumRecords + (1 << 32)
    else:
        raise ValueError(variant)
    return evs


def config_digest(name: str) -> str:
    """Fingerprint of a workloads.CONFIGS history (its collector JSONL), to
    detect a changed simulator."""
    import hashlib
    from s2_verification_amd import workloads as W
    return hashlib.sha256(W.config_jsonl(name)).hexdigest()[:32]
