"""CPU: s2Model.DescribeOperation / DescribeState strings (the labels of the
visualization page), pinned row by row against the reference's formats:
DescribeOperation main.go:341-352 with formatAppendCall main.go:363-406,
formatReadCall main.go:408-418, formatCheckTailCall main.go:420-426, and
DescribeState main.go:353-360. Every expected string below is the reference's
fmt.Sprintf format applied by hand to the op's fields."""
import s2_verification_amd as s2
from helpers import to_s2_events


def _ops():
    A = lambda i, n, hs, **kw: {"kind": "call", "op_id": i, "input_type": 0, "num_records": n, "record_hashes": hs, **kw}
    R = lambda i: {"kind": "call", "op_id": i, "input_type": 1}
    T = lambda i: {"kind": "call", "op_id": i, "input_type": 2}
    ok = lambda i, tail, **kw: {"kind": "return", "op_id": i, "failure": False, "definite_failure": False,
                                "tail": tail, **kw}
    fail = lambda i, definite: {"kind": "return", "op_id": i, "failure": True, "definite_failure": definite}
    rows = [
        # (call, return, expected DescribeOperation)
        (A(1, 1, [7]), ok(1, 1), "append(len[1], rh_last[7]) -> tail[1]"),
        (A(2, 2, [5, 9], set_fencing_token="tokA", match_seq_num=1), ok(2, 3),
         "append(len[2], set_token[tokA], match_seq_num[1], rh_last[9]) -> tail[3]"),
        (A(3, 1, [11], fencing_token="tokA"), fail(3, True),
         "append(len[1], batch_token[tokA], rh_last[11]) -> FAILED[definite]"),
        (A(4, 0, [], set_fencing_token="tokB", fencing_token="tokA"), fail(4, False),
         "append(len[0], set_token[tokB], batch_token[tokA]) -> FAILED[indefinite]"),
        (A(5, 3, [1, 2, 18446744073709551615], fencing_token="tokB", match_seq_num=4294967301), ok(5, 6),
         "append(len[3], batch_token[tokB], match_seq_num[4294967301], rh_last[18446744073709551615]) -> tail[6]"),
        (A(6, 1, [3], set_fencing_token=""), ok(6, 7), "append(len[1], set_token[], rh_last[3]) -> tail[7]"),
        (A(7, 0, []), ok(7, 7), "append(len[0]) -> tail[7]"),
        (R(8), ok(8, 7, stream_hash=42), "read() -> tail[7], hash[42]"),
        (R(9), ok(9, 7), "read() -> tail[7]"),  # (no StreamHash: expressible through the event API only)
        (R(10), fail(10, True), "read() -> failed"),
        (T(11), ok(11, 7), "check_tail() -> tail[7]"),
        (T(12), fail(12, True), "check_tail() -> failed"),
        (R(13), fail(13, False), "read() -> failed"),
    ]
    ev = []
    for c, r, _ in rows:
        ev += [c, r]
    return ev, [want for _, _, want in rows]


def test_describe_operation_matches_the_reference_formats():
    ev, want = _ops()
    h = s2.History.from_events(to_s2_events(ev))
    assert h.info()["n_ops"] == len(want)
    for d, w in enumerate(want):
        assert h.describe_operation(d) == w, (d, h.describe_operation(d), w)


def test_describe_operation_of_decoded_jsonl():
    """The same strings through the JSONL loader (collector serialization)."""
    jsonl = (
        b'{"event":{"Start":{"Append":{"num_records":2,"record_hashes":[5,9],"set_fencing_token":"tok",'
        b'"fencing_token":null,"match_seq_num":0}}},"client_id":1,"op_id":0}\n'
        b'{"event":{"Finish":{"AppendSuccess":{"tail":2}}},"client_id":1,"op_id":0}\n'
        b'{"event":{"Start":"Read"},"client_id":1,"op_id":1}\n'
        b'{"event":{"Finish":{"ReadSuccess":{"tail":2,"stream_hash":99}}},"client_id":1,"op_id":1}\n'
        b'{"event":{"Start":"CheckTail"},"client_id":2,"op_id":2}\n'
        b'{"event":{"Finish":"CheckTailFailure"},"client_id":2,"op_id":2}\n'
        b'{"event":{"Start":{"Append":{"num_records":1,"record_hashes":[4],"set_fencing_token":null,'
        b'"fencing_token":"tok","match_seq_num":null}}},"client_id":2,"op_id":3}\n'
        b'{"event":{"Finish":"AppendIndefiniteFailure"},"client_id":2,"op_id":3}\n'
        b'{"event":{"Start":"Read"},"client_id":1,"op_id":4}\n'
        b'{"event":{"Finish":"ReadFailure"},"client_id":1,"op_id":4}\n')
    h = s2.events_from_reader(jsonl)
    assert [h.describe_operation(d) for d in range(5)] == [
        "append(len[2], set_token[tok], match_seq_num[0], rh_last[9]) -> tail[2]",
        "read() -> tail[2], hash[99]",
        "check_tail() -> failed",
        "append(len[1], batch_token[tok], rh_last[4]) -> FAILED[indefinite]",
        "read() -> failed",
    ]


def test_describe_state_with_and_without_a_token():
    ev, _ = _ops()
    h = s2.History.from_events(to_s2_events(ev))
    assert h.describe_state((0, 0, 0)) == "tail[0],hash[0]"
    assert h.describe_state((18446744073709551615, 12345678901234567890, 0)) == \
        "tail[18446744073709551615],hash[12345678901234567890]"
    # a token-setting append's successor carries its token (an interned id)
    (s1,) = h.step((0, 0, 0), 0)
    (s2_,) = h.step(s1, 1)
    assert s2_[2] != 0
    assert h.describe_state(s2_) == "tail[3],hash[%d],token[tokA]" % s2_[1]
    # the empty-string token is a token (non-nil), printed empty
    (s3,) = h.step((6, 0, s2_[2]), 5)
    assert h.describe_state(s3) == "tail[7],hash[%d],token[]" % s3[1]


def test_describe_rejects_bad_arguments():
    ev, want = _ops()
    h = s2.History.from_events(to_s2_events(ev))
    import pytest
    with pytest.raises(s2.S2LCError):
        h.describe_operation(len(want))
    with pytest.raises(s2.S2LCError):
        h.describe_state((0, 0, 99))
