"""CPU: the binary SoA history cache (s2lc_history_save_many / load_many,
SURVEY.md §8f row 3): a decoded, finalized history survives the round trip
exactly (events, tokens, hashes, chains, the check's records), and a
malformed image is refused, never half-read.
"""
import os
import random
import struct

import pytest

import s2_verification_amd as s2
from helpers import GOLDEN, golden, random_history, to_s2_events


def _same(a, b):
    assert a.info() == b.info()
    assert a.events() == b.events()
    ea, eb = a.events_numpy(), b.events_numpy()
    # every field but the pointer-valued ones (record hashes, token strings)
    for f in ("kind", "op_id", "client_id", "input_type", "has_num_records", "has_match_seq_num", "num_records",
              "match_seq_num", "n_record_hashes", "failure", "definite_failure", "has_tail", "has_stream_hash",
              "tail", "stream_hash"):
        assert (ea[f] == eb[f]).all(), f


def _corpus():
    from s2_verification_amd import workloads as W
    hs = [s2.load_file(os.path.join(GOLDEN, c["jsonl_file"]))
          for c in golden("reference_cases.json")["cases"] if c.get("jsonl_file")]
    hs += [s2.History.from_events(to_s2_events(c["events"])) for c in golden("reference_cases.json")["cases"]]
    hs += W.c4_histories(60, first_seed=123)
    hs += [W.config_history(n) for n in ("C1", "C3")]
    rng = random.Random(5)
    hs += [s2.History.from_events(to_s2_events(random_history(rng, rng.randint(1, 9), 3))) for _ in range(60)]
    return hs


def test_round_trip_identity():
    hs = _corpus()
    img = s2.save_cache(hs)
    back = s2.load_cache(img)
    assert len(back) == len(hs)
    for a, b in zip(hs, back):
        _same(a, b)
    # an image of the loaded histories is the same bytes
    assert s2.save_cache(back) == img
    assert s2.load_cache(s2.save_cache([])) == []


def test_structural_and_event_only_histories_keep_every_event():
    """Histories whose events are not exactly call/return pairs (an unmatched
    call, a lone return) are stored with their whole event list."""
    unmatched = s2.events_from_reader(b'{"event":{"Start":"Read"},"client_id":1,"op_id":1}\n'
                                      b'{"event":{"Start":"CheckTail"},"client_id":2,"op_id":2}\n'
                                      b'{"event":{"Finish":{"CheckTailSuccess":{"tail":0}}},"client_id":2,"op_id":2}\n')
    lone = s2.events_from_reader(b'{"event":{"Finish":{"ReadSuccess":{"tail":7,"stream_hash":42}}},"client_id":1,"op_id":2}')
    assert unmatched.info()["structural"] != 0
    back = s2.load_cache(s2.save_cache([unmatched, lone]))
    _same(unmatched, back[0])
    _same(lone, back[1])


def test_loaded_histories_check_like_the_originals():
    """The check path reads only the cached records: verdicts through the CPU
    oracle of the loaded events, and the library's replay of a known order."""
    import oracle as orc
    hs = _corpus()[:40]
    back = s2.load_cache(s2.save_cache(hs))
    for a, b in zip(hs, back):
        va = orc.check_wgl(orc.from_s2lc_numpy(a.events_numpy()), timeout=10)[0]
        vb = orc.check_wgl(orc.from_s2lc_numpy(b.events_numpy()), timeout=10)[0]
        assert va == vb
        n = a.info()["n_ops"]
        if a.info()["structural"] == 0 and n:
            assert a.step((0, 0, 0), 0) == b.step((0, 0, 0), 0)


def test_malformed_images_are_refused():
    from s2_verification_amd import workloads as W
    img = s2.save_cache(W.c4_histories(3))
    bad = [b"", b"S2LCSOA0" + img[8:], img[:20], img[:len(img) // 2], img[:-8]]
    # an offset table pointing past the image
    n = struct.unpack_from("<Q", img, 16)[0]
    t = bytearray(img)
    struct.pack_into("<Q", t, 24 + 8 * n, len(img) * 4)
    bad.append(bytes(t))
    # a chain-start table that does not end at the record count
    t = bytearray(img)
    hdr = (24 + 8 * (n + 1) + 7) & ~7
    off0 = struct.unpack_from("<Q", img, 24)[0]
    struct.pack_into("<I", t, hdr + off0 + 16, 0xFFFFFF)  # K
    bad.append(bytes(t))
    for b in bad:
        with pytest.raises(s2.S2LCError) as e:
            s2.load_cache(b)
        assert e.value.status == -2
    # random corruption of the payload never crashes: refused or loaded
    rng = random.Random(3)
    for _ in range(200):
        t = bytearray(img)
        for _ in range(rng.randint(1, 8)):
            t[rng.randrange(hdr, len(t))] = rng.randrange(256)
        try:
            for h in s2.load_cache(bytes(t)):
                h.info()
                h.events()
        except s2.S2LCError as e:
            assert e.status == -2


def test_duplicate_id_histories_round_trip():
    """Duplicate-id histories (the literal engine's) are stored with their
    events and re-linked on load (History::finalize): same ops, same ids."""
    import random
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_literal import dup_history
    from helpers import to_s2_events
    rng = random.Random(3)
    hs = [s2.History.from_events(to_s2_events(dup_history(rng, 8, overlap=bool(k % 2)))) for k in range(6)]
    back = s2.load_cache(s2.save_cache(hs))
    for a, b in zip(hs, back):
        assert a.info() == b.info()
        ea, eb = a.events_numpy(), b.events_numpy()
        for f in ("kind", "op_id", "input_type", "num_records", "n_record_hashes", "failure", "tail", "stream_hash"):
            assert (ea[f] == eb[f]).all(), f


def test_wrapping_hash_range_is_refused():
    """An event whose record-hash range wraps the u64 sum (hash_off = 2^64 - 1,
    hash_cnt = 2: off + cnt = 1) must be refused, not handed out as a pointer
    past the pool (cache.cpp bounds checks)."""
    h = s2.events_from_reader(
        b'{"event":{"Start":{"Append":{"num_records":1,"record_hashes":[7],"set_fencing_token":null,'
        b'"fencing_token":null,"match_seq_num":null}}},"client_id":1,"op_id":1}\n')
    assert h.info()["structural"] != 0  # a call without a return: stored with its events (mode 1)
    img = s2.save_cache([h])
    assert s2.load_cache(img)[0].events() == h.events()
    hdr = (24 + 8 * 2 + 7) & ~7
    off0 = struct.unpack_from("<Q", img, 24)[0]
    ev0 = hdr + off0 + 72  # the section header is 72 bytes; Event (history.h): hash_off at +32, hash_cnt at +40
    assert struct.unpack_from("<QQ", img, ev0 + 32) == (0, 1)
    t = bytearray(img)
    struct.pack_into("<QQ", t, ev0 + 32, (1 << 64) - 1, 2)
    with pytest.raises(s2.S2LCError) as e:
        s2.load_cache(bytes(t))
    assert e.value.status == -2
