"""TEST INFRASTRUCTURE ONLY — Python face of the CPU oracle (oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (s2_verification_amd) never does.

Events are plain dicts in the porcupine.Event shape (golang/s2-porcupine/
main.go:206-225, 545-558):

    {"kind": "call"|"return", "op_id": int, "client_id": int,
     # call (StreamInput)
     "input_type": 0|1|2, "num_records": int|None, "match_seq_num": int|None,
     "set_fencing_token": str|None, "fencing_token": str|None, "record_hashes": [int],
     # return (StreamOutput)
     "failure": bool, "definite_failure": bool, "tail": int|None, "stream_hash": int|None}

``load_jsonl`` restates eventsFromReader (main.go:529-563) for well-formed
collector output using Python's json module; the product loader's edge cases
are pinned separately in tests/test_loader.py.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

OK, ILLEGAL, UNKNOWN, PANIC = 0, 1, 2, -2
_NAMES = {OK: "Ok", ILLEGAL: "Illegal", UNKNOWN: "Unknown", PANIC: "Panic", -1: "EInval"}

EVENT_DTYPE = np.dtype([
    ("kind", "<i4"), ("_pad0", "<i4"), ("op_id", "<i8"), ("client_id", "<i8"),
    ("input_type", "u1"), ("has_num_records", "u1"), ("has_msn", "u1"), ("_pad1", "u1"),
    ("set_tok", "<i4"), ("batch_tok", "<i4"), ("_pad2", "<i4"),
    ("num_records", "<u8"), ("msn", "<u8"), ("hashes", "<u8"), ("n_hashes", "<u8"),
    ("failure", "u1"), ("definite", "u1"), ("has_tail", "u1"), ("has_hash", "u1"), ("_pad3", "<u4"),
    ("tail", "<u8"), ("stream_hash", "<u8"),
])
assert EVENT_DTYPE.itemsize == 96


class _Stats(ctypes.Structure):
    _fields_ = [("cache_inserts", ctypes.c_uint64), ("steps", ctypes.c_uint64),
                ("backtracks", ctypes.c_uint64), ("max_state_set", ctypes.c_uint64),
                ("seconds", ctypes.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.or_chain_hash.restype = ctypes.c_uint64
        L.or_chain_hash.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_fold.restype = ctypes.c_uint64
        L.or_fold.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.or_check_wgl.restype = ctypes.c_int
        L.or_check_wgl.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double,
                                   ctypes.c_uint64, ctypes.POINTER(_Stats)]
        L.or_check_wgl_longest.restype = ctypes.c_int
        L.or_check_wgl_longest.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_uint64,
                                           ctypes.POINTER(_Stats), ctypes.c_void_p]
        L.or_check_reduced.restype = ctypes.c_int
        L.or_check_reduced.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Stats)]
        L.or_check_brute.restype = ctypes.c_int
        L.or_check_brute.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Stats)]
        _lib = L
    return _lib


def chain_hash(h: int, r: int) -> int:
    return lib().or_chain_hash(h, r)


def fold(h: int, rs) -> int:
    a = np.ascontiguousarray(np.asarray(rs, dtype=np.uint64))
    return lib().or_fold(h, a.ctypes.data, len(a))


class EventArray:
    """Events packed into the or_event layout (keeps the hash pool alive)."""

    def __init__(self, events):
        toks = {}

        def tok(s):
            if s is None:
                return 0
            return toks.setdefault(s, len(toks) + 1)

        n = len(events)
        arr = np.zeros(n, dtype=EVENT_DTYPE)
        pool = []
        offs = np.zeros(n, dtype=np.uint64)
        for i, e in enumerate(events):
            r = arr[i]
            call = e["kind"] == "call"
            r["kind"] = 0 if call else 1
            r["op_id"] = e["op_id"]
            r["client_id"] = e.get("client_id", 0)
            if call:
                r["input_type"] = e["input_type"]
                nr = e.get("num_records")
                r["has_num_records"] = nr is not None
                r["num_records"] = nr or 0
                msn = e.get("match_seq_num")
                r["has_msn"] = msn is not None
                r["msn"] = msn or 0
                r["set_tok"] = tok(e.get("set_fencing_token"))
                r["batch_tok"] = tok(e.get("fencing_token"))
                hs = e.get("record_hashes") or []
                offs[i] = len(pool)
                r["n_hashes"] = len(hs)
                pool.extend(hs)
            else:
                r["failure"] = bool(e.get("failure"))
                r["definite"] = bool(e.get("definite_failure"))
                t = e.get("tail")
                r["has_tail"] = t is not None
                r["tail"] = t or 0
                sh = e.get("stream_hash")
                r["has_hash"] = sh is not None
                r["stream_hash"] = sh or 0
        self.pool = np.array(pool, dtype=np.uint64) if pool else np.zeros(1, dtype=np.uint64)
        base = self.pool.ctypes.data
        arr["hashes"] = base + offs * 8
        self.arr = arr

    @property
    def ptr(self):
        return self.arr.ctypes.data

    def __len__(self):
        return len(self.arr)


def _as_array(events):
    return events if isinstance(events, EventArray) else EventArray(events)


def check_wgl(events, compute_partial=True, timeout=0.0, max_entries=0):
    """porcupine.CheckEventsVerbose(s2Model.ToModel(), events, timeout) restated."""
    ea = _as_array(events)
    st = _Stats()
    r = lib().or_check_wgl(ea.ptr, len(ea), int(compute_partial), float(timeout), int(max_entries),
                           ctypes.byref(st))
    return _NAMES[r], {"cache_inserts": st.cache_inserts, "steps": st.steps,
                       "backtracks": st.backtracks, "max_state_set": st.max_state_set,
                       "seconds": st.seconds}


def check_wgl_longest(events, timeout=0.0, max_entries=0):
    """LinearizationInfo's lengths: (verdict, [length of the longest partial
    linearization porcupine records containing dense op d, for d in 0..n-1])."""
    ea = _as_array(events)
    st = _Stats()
    n_ops = len(ea) // 2 + 1
    out = np.zeros(max(1, len(ea)), dtype=np.int32)
    r = lib().or_check_wgl_longest(ea.ptr, len(ea), float(timeout), int(max_entries), ctypes.byref(st),
                                   out.ctypes.data)
    return _NAMES[r], out


def check_brute(events):
    ea = _as_array(events)
    st = _Stats()
    r = lib().or_check_brute(ea.ptr, len(ea), ctypes.byref(st))
    return _NAMES[r], {"steps": st.steps}


def check_reduced(events, max_configs=0, reductions_off=0, round_counts=False):
    """CPU implementation of the GPU's reduced search (cross-check, not the reference).

    reductions_off: the product's RED_* bits; round_counts: also return the
    unique configurations of each completed round (stats["round_counts"])."""
    ea = _as_array(events)
    st = _Stats()
    cap = len(ea) + 2 if round_counts else 0
    rc = np.zeros(max(cap, 1), dtype=np.uint32)
    r = lib().or_check_reduced(ea.ptr, len(ea), int(max_configs), int(reductions_off),
                               rc.ctypes.data if round_counts else None, cap, ctypes.byref(st))
    out = {"configs": st.cache_inserts, "rounds": st.backtracks, "max_frontier": st.max_state_set,
           "children": st.steps, "seconds": st.seconds}
    if round_counts:
        out["round_counts"] = rc[:st.backtracks].tolist()
    return _NAMES[r], out


# ------------------------------------------------------------------ loader --
def _finish_to_output(fe):
    """outputFromFinish, main.go:466-523."""
    if isinstance(fe, str):
        if fe == "AppendDefiniteFailure":
            return dict(failure=True, definite_failure=True, tail=None, stream_hash=None)
        if fe == "AppendIndefiniteFailure":
            return dict(failure=True, definite_failure=False, tail=None, stream_hash=None)
        if fe in ("ReadFailure", "CheckTailFailure"):
            return dict(failure=True, definite_failure=True, tail=None, stream_hash=None)
        raise ValueError(f"unknown string finish event: {fe}")
    if not isinstance(fe, dict):
        raise ValueError("unknown finish event format")
    for k in ("AppendSuccess", "ReadSuccess", "CheckTailSuccess"):
        if k in fe:
            v = fe[k] or {}
            return dict(failure=False, definite_failure=False, tail=int(v.get("tail", 0)),
                        stream_hash=int(v.get("stream_hash", 0)) if k == "ReadSuccess" else None)
    raise ValueError("unknown finish event format")


def _start_to_input(se):
    """StartEvent.UnmarshalJSON + inputFromStart, main.go:32-70, 428-464."""
    if isinstance(se, str):
        if se == "Read":
            return dict(input_type=1)
        if se == "CheckTail":
            return dict(input_type=2)
        raise ValueError(f"unknown string start event: {se}")
    if isinstance(se, dict) and "Append" in se:
        a = se["Append"] or {}
        hs = [int(x) for x in (a.get("record_hashes") or [])]
        nr = int(a.get("num_records", 0))
        if len(hs) != nr:
            raise ValueError(f"append has {len(hs)} record_hashes but {nr} records")
        msn = a.get("match_seq_num")
        return dict(input_type=0, num_records=nr, record_hashes=hs,
                    set_fencing_token=a.get("set_fencing_token"),
                    fencing_token=a.get("fencing_token"),
                    match_seq_num=None if msn is None else int(msn))
    raise ValueError("unknown start event format")


def load_jsonl(text):
    """eventsFromReader restated for well-formed input (one JSON value per line)."""
    if isinstance(text, (bytes, bytearray)):
        text = text.decode()
    dec = json.JSONDecoder()
    events, i, n = [], 0, len(text)
    while True:
        while i < n and text[i] in " \t\r\n":
            i += 1
        if i >= n:
            return events
        rec, i = dec.raw_decode(text, i)
        ev = rec.get("event") or {}
        has_s, has_f = "Start" in ev, "Finish" in ev
        if has_s == has_f:
            raise ValueError("expected exactly one of Start/Finish")
        base = {"op_id": int(rec.get("op_id", 0)), "client_id": int(rec.get("client_id", 0))}
        if has_s:
            events.append({"kind": "call", **base, **_start_to_input(ev["Start"])})
        else:
            events.append({"kind": "return", **base, **_finish_to_output(ev["Finish"])})


def from_s2lc_numpy(ev, owner=None):
    """Product-exported events (numpy array in the s2lc_event layout, see
    s2_verification_amd.History.events_numpy) -> EventArray for the oracle.

    Token ids are re-derived from the exported string pointers (one pointer per
    distinct token string within a history). The exported record-hash pointers
    point into the source history: with `owner` (that history) the array keeps
    it alive and uses them as they are; without it the hashes are copied into a
    pool the array owns, so the source may be freed.
    """
    n = len(ev)
    arr = np.zeros(n, dtype=EVENT_DTYPE)
    for f_src, f_dst in (("kind", "kind"), ("op_id", "op_id"), ("client_id", "client_id"),
                         ("input_type", "input_type"), ("has_num_records", "has_num_records"),
                         ("has_match_seq_num", "has_msn"), ("num_records", "num_records"),
                         ("match_seq_num", "msn"), ("record_hashes", "hashes"), ("n_record_hashes", "n_hashes"),
                         ("failure", "failure"), ("definite_failure", "definite"), ("has_tail", "has_tail"),
                         ("has_stream_hash", "has_hash"), ("tail", "tail"), ("stream_hash", "stream_hash")):
        arr[f_dst] = ev[f_src]
    ptrs = np.concatenate([ev["set_fencing_token"], ev["fencing_token"]])
    uniq, inv = np.unique(ptrs, return_inverse=True)
    ids = inv.astype(np.int32) + (0 if uniq[0] == 0 else 1)  # pointer 0 (nil) -> id 0
    arr["set_tok"] = ids[:n]
    arr["batch_tok"] = ids[n:]
    ea = EventArray.__new__(EventArray)
    ea.arr = arr
    ea.pool = owner
    if owner is None:
        cnt = arr["n_hashes"].astype(np.int64)
        has = np.nonzero(cnt)[0]
        offs = np.zeros(n, dtype=np.int64)
        offs[has] = np.cumsum(cnt[has]) - cnt[has]
        pool = np.zeros(max(1, int(cnt.sum())), dtype=np.uint64)
        base = pool.ctypes.data
        for i in has.tolist():
            ctypes.memmove(base + 8 * int(offs[i]), int(arr["hashes"][i]), 8 * int(cnt[i]))
        arr["hashes"] = np.where(cnt > 0, base + offs * 8, 0).astype(arr["hashes"].dtype)
        ea.pool = pool
    return ea
