"""CPU: the product JSONL loader (eventsFromReader, main.go:529-563 semantics)."""
import json
import os

import pytest

import s2_verification_amd as s2
from helpers import GOLDEN, golden, from_s2_events


def load(text):
    return s2.events_from_reader(text)


def decode_fails(text):
    with pytest.raises(s2.S2LCError) as ei:
        load(text)
    assert ei.value.status == -2
    return str(ei.value)


def test_rejects_malformed_json():
    """TestEventsFromReaderRejectsMalformedJSON (main_test.go:103-108)."""
    decode_fails('{"event":{"Start":"Read"},"client_id":1,"op_id":1')


def test_read_success_stream_hash():
    """TestEventsFromReaderDecodesReadSuccessStreamHash (main_test.go:110-126)."""
    h = load('{"event":{"Finish":{"ReadSuccess":{"tail":7,"stream_hash":42}}},"client_id":1,"op_id":2}')
    ev = h.events()
    assert len(ev) == 1
    assert ev[0].Value.StreamHash == 42 and ev[0].Value.Tail == 7


def test_large_record_hash_line():
    """TestEventsFromReaderHandlesLargeRecordHashLine (main_test.go:34-101): >64 KiB line, exact u64s."""
    with open(os.path.join(GOLDEN, "ref_LargeRecordHashLine.jsonl"), "rb") as f:
        data = f.read()
    assert data.index(b"\n") > 64 * 1024
    ev = load(data).events()
    assert len(ev) == 2
    assert ev[0].Value.RecordHashes == [2**64 - 1 - i for i in range(5000)]


def test_golden_files_match_fixture_events():
    for c in golden("reference_cases.json")["cases"]:
        if not c.get("jsonl_file"):
            continue
        got = from_s2_events(s2.load_file(os.path.join(GOLDEN, c["jsonl_file"])).events())
        want = c["events"]
        assert len(got) == len(want)
        for g, w in zip(got, want):
            for k, v in w.items():
                if k == "client_id":
                    continue
                assert g.get(k) == v, (c["name"], k, g, w)


def test_num_records_mismatch():
    decode_fails('{"event":{"Start":{"Append":{"num_records":2,"record_hashes":[1],'
                 '"set_fencing_token":null,"fencing_token":null,"match_seq_num":null}}},"client_id":1,"op_id":1}')


@pytest.mark.parametrize("text", [
    '{"event":{"Start":"Write"},"client_id":1,"op_id":1}',                 # unknown string start
    '{"event":{"Start":{"Foo":{}}},"client_id":1,"op_id":1}',              # unknown start object
    '{"event":{"Start":5},"client_id":1,"op_id":1}',                       # number start
    '{"event":{"Finish":"Boom"},"client_id":1,"op_id":1}',                 # unknown finish
    '{"event":{"Finish":{"Nope":{}}},"client_id":1,"op_id":1}',            # unknown finish object
    '{"event":{"Start":"Read","Finish":"ReadFailure"},"client_id":1,"op_id":1}',  # both
    '{"event":{},"client_id":1,"op_id":1}',                                # neither
    '{"event":null,"client_id":1,"op_id":1}',                              # null event
    '{"client_id":1,"op_id":1}',                                           # no event
    'null',                                                                # null record
    '[1,2]',                                                               # array record
    '{"event":{"Start":"Read"},"client_id":"1","op_id":1}',                # string id
    '{"event":{"Start":"Read"},"client_id":1,"op_id":1.5}',                # fractional id
    '{"event":{"Start":"Read"},"client_id":1,"op_id":1e3}',                # exponent id
    '{"event":{"Start":{"Append":{"num_records":-1,"record_hashes":[]}}},"op_id":1}',  # negative u64
    '{"event":{"Start":{"Append":{"num_records":18446744073709551616,"record_hashes":[]}}},"op_id":1}',
    '{"event":{"Start":{"Append":{"num_records":0,"record_hashes":[],"set_fencing_token":5}}},"op_id":1}',
    '{"event":{"Finish":{"AppendSuccess":{"tail":"4"}}},"op_id":1}',
    '{"event":{"Start":"Read"},"op_id":01}',                               # leading zero
    '{"event":{"Start":"Read"}} x',                                        # trailing garbage
    '{"event":{"Start":"Read"},"event":{"Finish":"ReadFailure"},"op_id":1}',  # duplicate event key accumulates
    '{"event":{"Start":"Re\\x"},"op_id":1}',                               # bad escape
])
def test_decode_errors(text):
    decode_fails(text)


def test_go_decoder_leniencies():
    # case-insensitive struct keys, unknown keys ignored, null ids, any whitespace, no newlines needed
    h = load('  {"EVENT":{"Start":"CheckTail"},"Client_Id":3,"OP_ID":9,"extra":[1,{"a":null}]}'
             '{"event":{"Finish":{"CheckTailSuccess":{"TAIL":5,"junk":true}}},"client_id":null,"op_id":9}\n\n')
    ev = h.events()
    assert [e.Kind for e in ev] == [0, 1]
    assert ev[0].Id == 9 and ev[0].ClientId == 3 and ev[0].Value.InputType == 2
    assert ev[1].Value.Tail == 5 and ev[1].ClientId == 0
    # Kelvin sign / long s fold like ASCII k / s in struct keys (Go encoding/json)
    h = load('{"event":{"Start":{"Append":{"num_recordſ":1,"record_hashes":[7],'
             '"fencing_toKen":"t"}}},"op_id":1}'.encode("utf-8"))
    v = h.events()[0].Value
    assert v.NumRecords == 1 and v.BatchFencingToken == "t"
    # map keys ("Start", "Append", ...) are exact
    decode_fails('{"event":{"start":"Read"},"op_id":1}')
    # duplicate keys: last wins (maps and struct fields)
    h = load('{"event":{"Start":"Read","Start":"CheckTail"},"op_id":1,"op_id":4}')
    assert h.events()[0].Value.InputType == 2 and h.events()[0].Id == 4
    # null Append payload = zero AppendArgs; null success payload = zero result
    h = load('{"event":{"Start":{"Append":null}},"op_id":1}{"event":{"Finish":{"AppendSuccess":null}},"op_id":1}')
    ev = h.events()
    assert ev[0].Value.NumRecords == 0 and ev[1].Value.Tail == 0
    # record_hashes null elements decode as 0; escapes decode
    h = load('{"event":{"Start":{"Append":{"num_records":2,"record_hashes":[null,3],'
             '"set_fencing_token":"\\u0041b"}}},"op_id":1}')
    v = h.events()[0].Value
    assert v.RecordHashes == [0, 3] and v.SetFencingToken == "Ab"
    # empty input: no events
    assert len(load("")) == 0
    # string Start "Read" with unicode escape
    assert load('{"event":{"Start":"Re\\u0061d"},"op_id":1}').events()[0].Value.InputType == 1


def test_append_failure_mapping():
    """outputFromFinish (main.go:466-523)."""
    rows = {
        '"AppendDefiniteFailure"': (True, True, None, None),
        '"AppendIndefiniteFailure"': (True, False, None, None),
        '"ReadFailure"': (True, True, None, None),
        '"CheckTailFailure"': (True, True, None, None),
        '{"AppendSuccess":{"tail":3}}': (False, False, 3, None),
        '{"ReadSuccess":{"tail":3,"stream_hash":9}}': (False, False, 3, 9),
        '{"CheckTailSuccess":{"tail":3}}': (False, False, 3, None),
        '{"ReadSuccess":{}}': (False, False, 0, 0),
    }
    for fin, want in rows.items():
        v = load('{"event":{"Finish":%s},"op_id":1}' % fin).events()[0].Value
        assert (v.Failure, v.DefiniteFailure, v.Tail, v.StreamHash) == want, fin


def test_simulator_jsonl_roundtrip():
    """The simulator's JSONL and its direct history agree event for event."""
    for wf in (0, 1, 2):
        data = s2.simulate_jsonl(workflow=wf, num_clients=4, ops_per_client=50, seed=11, p_indefinite=0.05)
        a = from_s2_events(load(data).events())
        b = from_s2_events(s2.simulate_history(workflow=wf, num_clients=4, ops_per_client=50, seed=11,
                                               p_indefinite=0.05).events())
        assert a == b
        # serde field order (history.rs:133-138)
        first = json.loads(data.split(b"\n")[0])
        assert list(first.keys()) == ["event", "client_id", "op_id"]


def test_load_many_parallel_equals_sequential():
    """s2lc_load_jsonl_many (threads) decodes each buffer exactly like s2lc_load_jsonl."""
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    blobs = [s2.simulate_jsonl(**W.c4_params(seed)) for seed in range(40)]
    many = s2.load_many(blobs, threads=4)
    for b, h in zip(blobs, many):
        one = s2.events_from_reader(b)
        assert h.info() == one.info()
        assert h.events() == one.events()


def test_load_many_reports_first_bad_buffer():
    import pytest
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    blobs = [s2.simulate_jsonl(**W.c4_params(seed)) for seed in range(6)]
    blobs[4] = b'{"event":{"Start":"Read"},"client_id":1'
    blobs[2] = blobs[2] + b"not json\n"
    with pytest.raises(s2.S2LCError) as e:
        s2.load_many(blobs, threads=3)
    assert "history 2:" in str(e.value)


def _canon_or_error(data):
    try:
        h = load(data)
    except s2.S2LCError as e:
        return ("error", e.status, str(e))
    return ("ok", h.info()["n_events"], [(e.Kind, e.Id, e.ClientId, repr(e.Value)) for e in h.events()])


def _perturbations(text):
    """Variants of a collector-format blob that leave the fast path's form
    (the general parser takes those records) or are invalid."""
    lines = text.splitlines(keepends=True)
    out = []
    for i in range(0, min(len(lines), 40), 7):
        ln = lines[i]
        for a, b in (('":', '": '), ('"event"', '"Event"'), ('"client_id":', '"client_id":-'),
                     ('"op_id":', '"op_id":0'), ('"tail":', '"tail":1.5e'), ('"num_records":', '"num_records":1'),
                     ('"set_fencing_token":null', '"set_fencing_token":"t\\u00e9"'),
                     ('"fencing_token":null', '"fencing_token":"éx"'), (',"op_id"', ',"x":[1,2],"op_id"'),
                     ('}\n', '}  '), ('{"event"', '\t{"event"'), ('"Read"', '"Re\\u0061d"'),
                     ('"match_seq_num":null', '"match_seq_num":7'), ('[', '[ ')):
            if a in ln:
                out.append("".join(lines[:i] + [ln.replace(a, b, 1)] + lines[i + 1:]))
    return out


def test_fast_path_decodes_like_the_general_parser(monkeypatch):
    """jsonl.cpp decodes records in the collector's exact serialisation without
    a JSON tree and hands every other record to the general (Go encoding/json)
    parser: same events, tokens and errors either way (S2LC_JSONL_GENERAL=1
    forces the general parser)."""
    from s2_verification_amd import workloads as W
    blobs = [open(os.path.join(GOLDEN, f), "rb").read().decode() for f in sorted(os.listdir(GOLDEN))
             if f.endswith(".jsonl")]
    blobs += [s2.simulate_jsonl(**W.c4_params(sd)).decode() for sd in range(0, 30)]
    blobs.append(W.config_jsonl("C3").decode())
    cases = list(blobs)
    for b in blobs[:12] + blobs[-3:]:
        cases += _perturbations(b)
    assert len(cases) > 150
    n_err = 0
    for data in cases:
        monkeypatch.delenv("S2LC_JSONL_GENERAL", raising=False)
        fast = _canon_or_error(data.encode("utf-8"))
        monkeypatch.setenv("S2LC_JSONL_GENERAL", "1")
        general = _canon_or_error(data.encode("utf-8"))
        assert fast == general, data[:300]
        n_err += fast[0] == "error"
    assert 0 < n_err < len(cases)


def test_fast_path_integers_at_every_length(monkeypatch):
    """The fast path parses a digit run as right-aligned 8-digit groups (and
    bounds a 20-digit one arithmetically): every length 1..20, the uint64 /
    int64 limits and one past them decode (or fail) as the general parser does."""
    vals = ["0", "01", "00"]
    for k in range(1, 21):
        vals += [str(10 ** k - 1), str(10 ** (k - 1)), "1234567890123456789012"[:k]]
    vals += ["18446744073709551615", "18446744073709551616", "18446744073709551625", "18446744073709552615",
             "18440000000000000000", "18449999999999999999", "18450000000000000000", "99999999999999999999",
             "184467440737095516150", "9223372036854775807", "9223372036854775808"]
    n_err = 0
    for v in vals:
        for where in ("hash", "tail", "client", "op"):
            h = v if where == "hash" else "5"
            t = v if where == "tail" else "3"
            c = v if where == "client" else "1"
            o = v if where == "op" else "0"
            data = ('{"event":{"Start":{"Append":{"num_records":1,"record_hashes":[%s],"set_fencing_token":null,'
                    '"fencing_token":null,"match_seq_num":%s}}},"client_id":%s,"op_id":%s}\n'
                    '{"event":{"Finish":{"ReadSuccess":{"tail":%s,"stream_hash":%s}}},"client_id":%s,"op_id":%s}\n'
                    % (h, t, c, o, t, h, c, o)).encode()
            monkeypatch.delenv("S2LC_JSONL_GENERAL", raising=False)
            fast = _canon_or_error(data)
            monkeypatch.setenv("S2LC_JSONL_GENERAL", "1")
            general = _canon_or_error(data)
            assert fast == general, (v, where)
            n_err += fast[0] == "error"
    assert 0 < n_err < 4 * len(vals)


@pytest.mark.parametrize("general", [False, True])
def test_many_distinct_fencing_tokens(monkeypatch, general):
    """A history with thousands of distinct fencing tokens (one per append)
    interns each once and maps every event back to its own string, through
    both decoders; reused tokens keep their first id (the number of distinct
    tokens, n_tokens, counts each once)."""
    import time
    if general:
        monkeypatch.setenv("S2LC_JSONL_GENERAL", "1")
    n = 6000
    lines = []
    for i in range(n):
        lines.append('{"event":{"Start":{"Append":{"num_records":0,"record_hashes":[],"set_fencing_token":"s%d",'
                     '"fencing_token":%s,"match_seq_num":null}}},"client_id":1,"op_id":%d}'
                     % (i, '"s%d"' % (i // 2) if i % 3 else "null", i))
        lines.append('{"event":{"Finish":"AppendDefiniteFailure"},"client_id":1,"op_id":%d}' % i)
    t0 = time.perf_counter()
    h = load("\n".join(lines).encode())
    assert time.perf_counter() - t0 < 5.0  # (a scan per token: ~18 M string compares)
    evs = h.events()
    for i in range(n):
        v = evs[2 * i].Value
        assert v.SetFencingToken == "s%d" % i
        assert v.BatchFencingToken == ("s%d" % (i // 2) if i % 3 else None)
    assert h.info()["n_tokens"] == n


def _structural_variants(text):
    """Collector-form blobs the direct decode must hand to load_jsonl + finalize:
    op ids not 0, 1, 2, ... in call order, a second Finish, an op never
    returned, a Finish before its Start."""
    lines = text.splitlines(keepends=True)
    out = [text.replace('"op_id":', '"op_id":1', 1)]  # first op id 10.. (not dense)
    fin = [i for i, ln in enumerate(lines) if '"Finish"' in ln]
    if fin:
        out.append("".join(lines + [lines[fin[len(fin) // 2]]]))  # a second Finish
        out.append("".join(lines[:fin[-1]] + lines[fin[-1] + 1:]))  # an op never returned
        i = fin[0]
        out.append("".join([lines[i]] + lines[:i] + lines[i + 1:]))  # a Finish before its Start
    return out


def test_direct_decode_leaves_the_finalized_state(monkeypatch):
    """load_jsonl_finalized decodes a history in the collector's form straight
    into the finalized records, chains and op tables (events built on first
    use). It must leave exactly what load_jsonl + History::finalize leave
    (S2LC_JSONL_DIRECT=0): the same info, events and byte-identical cache
    images (records with their P1 bounds, chain starts, op tables, pool, tokens,
    client ids), over C4 and workflow histories, > 32 chains (the colouring's
    heap), fencing tokens, and the structural variants it hands back to the
    general path."""
    from s2_verification_amd import workloads as W
    blobs = [s2.simulate_jsonl(**W.c4_params(sd)) for sd in range(0, 24)]
    for wf in (0, 1, 2):
        blobs.append(s2.simulate_jsonl(workflow=wf, num_clients=5, ops_per_client=60, seed=3 + wf, p_indefinite=0.1))
    blobs.append(s2.simulate_jsonl(workflow=0, num_clients=48, ops_per_client=12, seed=9, p_indefinite=0.05))
    blobs += [open(os.path.join(GOLDEN, f), "rb").read() for f in sorted(os.listdir(GOLDEN)) if f.endswith(".jsonl")]
    cases = list(blobs)
    for b in blobs[:4] + blobs[24:28]:
        cases += [v.encode() for v in _structural_variants(b.decode())]
    many_chains = 0
    for data in cases:
        got = {}
        for mode in ("1", "0"):
            monkeypatch.setenv("S2LC_JSONL_DIRECT", mode)
            try:
                h = load(data)
            except s2.S2LCError as e:
                got[mode] = ("error", e.status, str(e))
                continue
            got[mode] = ("ok", h.info(), [(e.Kind, e.Id, e.ClientId, repr(e.Value)) for e in h.events()],
                         s2.save_cache([h]))
            if mode == "1" and h.info()["n_chains"] > 32:
                many_chains += 1
        assert got["1"] == got["0"], data[:200]
    assert many_chains >= 1


def test_history_pool_trim():
    """Released histories are parked for the next decode (S2LC_HISTORY_POOL_MB,
    accounted by array capacity); s2lc_history_pool_trim returns them to the
    heap and reports the bytes, and decoding afterwards is unchanged."""
    import gc
    from s2_verification_amd import workloads as W
    blobs = [s2.simulate_jsonl(**W.c4_params(sd)) for sd in range(8)]
    want = [h.events() for h in s2.load_many(blobs, threads=2)]
    gc.collect()
    s2.history_pool_trim()
    hs = s2.load_many(blobs, threads=2)
    n_bytes = sum(len(b) for b in blobs)
    del hs
    gc.collect()
    freed = s2.history_pool_trim()
    assert n_bytes // 4 < freed < 4 * n_bytes  # records, pool, op tables: ~0.7x the JSONL
    assert s2.history_pool_trim() == 0
    assert [h.events() for h in s2.load_many(blobs, threads=2)] == want
