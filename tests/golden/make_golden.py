"""Generates the committed golden fixtures in tests/golden/ (run here, not on the GPU box).

Sources (data only — no reference source text is copied):
  * chain_hash_vectors.json — the reference's chain-hash known answers
    (golang/s2-porcupine/main_test.go:15-32, rust/s2-verification/src/history.rs:678-687)
    plus random (h, r) pairs hashed by python-xxhash 3.8.1 (libxxhash 0.8.2), an
    independent XXH3 implementation of what zeebo/xxh3 HashSeed computes
    (main.go:232-236).
  * reference_cases.json — the reference's verdict tests (main_test.go:34-400)
    re-expressed as porcupine event lists with their expected verdicts. The
    record hashes / cumulative stream hashes the tests compute with
    foldRecordHashes are recomputed here with python-xxhash.
  * ref_*.jsonl — the same cases in collector JSONL form where JSONL can express
    them (the NumRecords=2^32+5-with-one-hash case cannot: the loader rejects it,
    main.go:62-64).

Usage: python tests/golden/make_golden.py
"""
import json
import os
import random

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))


def chain_hash(h, r):
    return xxhash.xxh3_64_intdigest(r.to_bytes(8, "little"), seed=h)


def fold(h, rs):
    for r in rs:
        h = chain_hash(h, r)
    return h


def hash_vectors():
    foo = xxhash.xxh3_64_intdigest(b"foo")
    bar = xxhash.xxh3_64_intdigest(b"bar")
    baz = xxhash.xxh3_64_intdigest(b"baz")
    h1 = chain_hash(0, foo)
    h2 = chain_hash(h1, bar)
    h3 = chain_hash(h2, baz)
    ref = {"xxh3_foo": 0xab6e5f64077e7d8a, "h1": 0x4d2b003ee417c3a5,
           "h2": 0x132e5d5dd7936edd, "h3": 0x732ee99abc5002ff}
    assert (foo, h1, h2, h3) == (ref["xxh3_foo"], ref["h1"], ref["h2"], ref["h3"]), "xxhash disagrees with reference KAT"
    rng = random.Random(20261015)
    pairs = []
    specials = [0, 1, 2**32 - 1, 2**32, 2**63, 2**64 - 1, 0x0123456789ABCDEF]
    for h in specials:
        for r in specials:
            pairs.append([h, r, chain_hash(h, r)])
    for _ in range(400):
        h, r = rng.getrandbits(64), rng.getrandbits(64)
        pairs.append([h, r, chain_hash(h, r)])
    folds = []
    for _ in range(40):
        h = rng.getrandbits(64) if rng.random() < 0.5 else 0
        rs = [rng.getrandbits(64) for _ in range(rng.randint(0, 17))]
        folds.append([h, rs, fold(h, rs)])
    return {
        "source": "main_test.go:15-32 / history.rs:678-687 + python-xxhash 3.8.1 xxh3_64(le64(r), seed=h)",
        "reference": {"inputs": ["foo", "bar", "baz"], "xxh3": [foo, bar, baz], **ref},
        "pairs": pairs,
        "folds": folds,
    }


# ---------------------------------------------------------------- cases ---
def call_append(op, batch, num=None, msn=None, set_tok=None, tok=None, client=0):
    return {"kind": "call", "op_id": op, "client_id": client, "input_type": 0,
            "num_records": len(batch) if num is None else num, "record_hashes": list(batch),
            "match_seq_num": msn, "set_fencing_token": set_tok, "fencing_token": tok}


def call_read(op, client=0):
    return {"kind": "call", "op_id": op, "client_id": client, "input_type": 1}


def call_check_tail(op, client=0):
    return {"kind": "call", "op_id": op, "client_id": client, "input_type": 2}


def ret(op, failure=False, definite=False, tail=None, stream_hash=None, client=0):
    return {"kind": "return", "op_id": op, "client_id": client, "failure": failure,
            "definite_failure": definite, "tail": tail, "stream_hash": stream_hash}


def reference_cases():
    cases = []

    def add(name, src, expected, events, jsonl=True):
        cases.append({"name": name, "source": src, "expected": expected, "jsonl": jsonl, "events": events})

    # TestEventsFromReaderHandlesLargeRecordHashLine (main_test.go:34-101)
    big = [2**64 - 1 - i for i in range(5000)]
    add("LargeRecordHashLine", "main_test.go:34-101", "Ok",
        [call_append(0, big), ret(0, tail=5000)])

    b1 = [11, 22, 33, 44]
    b2 = [55, 66, 77, 88, 99]
    h1 = fold(0, b1)
    h2 = fold(h1, b2)
    prefix = [call_append(0, b1), ret(0, tail=4),
              call_read(1), ret(1, tail=4, stream_hash=h1),
              call_check_tail(2), ret(2, tail=4)]
    # TestBasicNoConcurrency (main_test.go:128-152)
    add("BasicNoConcurrency", "main_test.go:128-152", "Ok", prefix)
    # TestBasicNoConcurrencyDefiniteFailure1 (main_test.go:154-191)
    add("DefiniteFailure1", "main_test.go:154-191", "Ok", prefix + [
        call_append(3, b2), ret(3, failure=True, definite=True),
        call_read(4), ret(4, tail=4, stream_hash=h1)])
    # TestBasicNoConcurrencyDefiniteFailure2 (main_test.go:192-232)
    add("DefiniteFailure2", "main_test.go:192-232", "Illegal", prefix + [
        call_append(3, b2), ret(3, failure=True, definite=True),
        call_read(4), ret(4, tail=9, stream_hash=h2)])
    # TestBasicNoConcurrencyIndefiniteFailure1 (main_test.go:233-272)
    add("IndefiniteFailure1", "main_test.go:233-272", "Ok", prefix + [
        call_append(3, b2), ret(3, failure=True),
        call_read(4), ret(4, tail=9, stream_hash=h2)])
    # TestBasicNoConcurrencyIndefiniteFailure2 (main_test.go:273-311)
    add("IndefiniteFailure2", "main_test.go:273-311", "Ok", prefix + [
        call_append(3, b2), ret(3, failure=True),
        call_read(4), ret(4, tail=4, stream_hash=h1)])
    # TestLargeSeqNumsNotTruncated (main_test.go:315-343): NumRecords 2^32+5 with one hash
    big_tail = 2**32 + 5
    add("LargeSeqNums_msn5", "main_test.go:315-335", "Illegal", [
        call_append(0, [11], num=big_tail), ret(0, tail=big_tail),
        call_append(1, [22], num=1, msn=5), ret(1, tail=big_tail + 1)], jsonl=False)
    add("LargeSeqNums_msnBig", "main_test.go:337-342", "Ok", [
        call_append(0, [11], num=big_tail), ret(0, tail=big_tail),
        call_append(1, [22], num=1, msn=big_tail), ret(1, tail=big_tail + 1)], jsonl=False)
    # TestReadDetectsCorruptedPrefix (main_test.go:349-374)
    c1, c2 = [11, 22], [33]
    h_corrupt = fold(fold(0, [98, 99]), c2)
    add("ReadDetectsCorruptedPrefix", "main_test.go:349-374", "Illegal", [
        call_append(0, c1), ret(0, tail=2), call_append(1, c2), ret(1, tail=3),
        call_read(2), ret(2, tail=3, stream_hash=h_corrupt)])
    # TestReadVerifiesWholeStream (main_test.go:378-400)
    h_ok = fold(fold(0, c1), c2)
    add("ReadVerifiesWholeStream", "main_test.go:378-400", "Ok", [
        call_append(0, c1), ret(0, tail=2), call_append(1, c2), ret(1, tail=3),
        call_read(2), ret(2, tail=3, stream_hash=h_ok)])
    return cases


def to_jsonl(events):
    """Collector serde form (history.rs:85-138; field order event, client_id, op_id)."""
    lines = []
    for e in events:
        if e["kind"] == "call":
            t = e["input_type"]
            if t == 1:
                start = "Read"
            elif t == 2:
                start = "CheckTail"
            else:
                start = {"Append": {"num_records": e["num_records"], "record_hashes": e["record_hashes"],
                                    "set_fencing_token": e["set_fencing_token"],
                                    "fencing_token": e["fencing_token"], "match_seq_num": e["match_seq_num"]}}
            ev = {"Start": start}
        else:
            ev = {"Finish": e["_finish"]}  # set by annotate_finish()
        lines.append(json.dumps({"event": ev, "client_id": e["client_id"], "op_id": e["op_id"]},
                                separators=(",", ":")))
    return "\n".join(lines) + "\n"


def annotate_finish(events):
    """Attach the collector Finish variant each return came from (CallFinish, history.rs:100-118)."""
    kind_of = {}
    for e in events:
        if e["kind"] == "call":
            kind_of[e["op_id"]] = e["input_type"]
        else:
            t = kind_of[e["op_id"]]
            if t == 0:
                if e["failure"]:
                    e["_finish"] = "AppendDefiniteFailure" if e["definite_failure"] else "AppendIndefiniteFailure"
                else:
                    e["_finish"] = {"AppendSuccess": {"tail": e["tail"]}}
            elif t == 1:
                e["_finish"] = "ReadFailure" if e["failure"] else {
                    "ReadSuccess": {"tail": e["tail"], "stream_hash": e["stream_hash"]}}
            else:
                e["_finish"] = "CheckTailFailure" if e["failure"] else {"CheckTailSuccess": {"tail": e["tail"]}}


def main():
    with open(os.path.join(HERE, "chain_hash_vectors.json"), "w") as f:
        json.dump(hash_vectors(), f, indent=0)
    cases = reference_cases()
    for c in cases:
        if c["jsonl"]:
            annotate_finish(c["events"])
            path = os.path.join(HERE, f"ref_{c['name']}.jsonl")
            with open(path, "w") as f:
                f.write(to_jsonl(c["events"]))
            c["jsonl_file"] = os.path.basename(path)
            for e in c["events"]:
                e.pop("_finish", None)
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump({"source": "golang/s2-porcupine/main_test.go (verdict tests)", "cases": cases}, f)
    print(f"wrote {len(cases)} reference cases")


if __name__ == "__main__":
    main()
