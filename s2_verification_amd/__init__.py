"""s2_verification_amd — MI355X linearizability checker for the S2 stream model.

Python face of libs2lincheck (include/s2lincheck.h), mirroring the reference's
Go surface so callers and tests read like golang/s2-porcupine/main_test.go:

    reference (Go)                                  here
    ----------------------------------------------  ------------------------------------
    StreamInput / StreamOutput   main.go:206-225     StreamInput / StreamOutput
    porcupine.Event{Kind,Value,Id,ClientId}          Event(kind, value, id, client_id)
    porcupine.CallEvent / ReturnEvent                CallEvent / ReturnEvent
    eventsFromReader(r)          main.go:529-563     events_from_reader(data) -> History
    chainHash / foldRecordHashes main.go:227-244     chain_hash / fold_record_hashes
    porcupine.CheckEventsVerbose main.go:606         check_events_verbose(model, events, timeout)
    porcupine.Ok / Illegal / Unknown                 Ok / Illegal / Unknown

The check itself only runs on the GPU (HIP, gfx950). Without a device
``Checker()`` raises; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("S2LC_LIB") or os.path.join(_HERE, "libs2lincheck.so")
CLI_PATH = os.path.join(_HERE, "s2-porcupine")

# ------------------------------------------------------------------ C ABI ---
S2LC_OK, S2LC_ILLEGAL, S2LC_UNKNOWN = 0, 1, 2
CallEvent, ReturnEvent = 0, 1
Ok, Illegal, Unknown = "Ok", "Illegal", "Unknown"
_VERDICT = {S2LC_OK: Ok, S2LC_ILLEGAL: Illegal, S2LC_UNKNOWN: Unknown}
STATUS = {0: "SUCCESS", -1: "EINVAL", -2: "EDECODE", -3: "EIO", -4: "ENODEV", -5: "EHIP",
          -6: "EUNSUPPORTED", -7: "ENOMEM", -8: "EWITNESS"}
EWITNESS = -8
REASONS = {0: "none", 1: "unmatched", 2: "search_exhausted", 3: "budget", 4: "frontier", 5: "witness_invalid",
           6: "timeout"}
# s2lc_engine: force a search engine (tests / diagnostics)
ENGINE_AUTO, ENGINE_WORKGROUP, ENGINE_WORKGROUP_HBM, ENGINE_LEVEL = 0, 1, 2, 3
# S2LC_RED_*: verdict-exact search reductions that can be disabled (ablation tests)
RED_P1, RED_P2, RED_P4, RED_IDEFER = 0x1, 0x2, 0x4, 0x8
F_NO_WITNESS, F_ROUND_COUNTS = 0x1, 0x2
WF_REGULAR, WF_MATCH_SEQ_NUM, WF_FENCING = 0, 1, 2
VIOL_NONE, VIOL_READ_HASH, VIOL_DEFINITE_APPLIED, VIOL_TAIL, VIOL_STALE_MSN = 0, 1, 2, 3, 4


class S2LCError(RuntimeError):
    def __init__(self, status, msg=""):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status


class c_event(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32), ("op_id", ctypes.c_int64), ("client_id", ctypes.c_int64),
        ("input_type", ctypes.c_uint8), ("has_num_records", ctypes.c_uint8),
        ("has_match_seq_num", ctypes.c_uint8), ("_pad0", ctypes.c_uint8),
        ("num_records", ctypes.c_uint64), ("match_seq_num", ctypes.c_uint64),
        ("set_fencing_token", ctypes.c_char_p), ("fencing_token", ctypes.c_char_p),
        ("record_hashes", ctypes.POINTER(ctypes.c_uint64)), ("n_record_hashes", ctypes.c_uint64),
        ("failure", ctypes.c_uint8), ("definite_failure", ctypes.c_uint8), ("has_tail", ctypes.c_uint8),
        ("has_stream_hash", ctypes.c_uint8), ("_pad1", ctypes.c_uint32),
        ("tail", ctypes.c_uint64), ("stream_hash", ctypes.c_uint64),
    ]


class c_state(ctypes.Structure):
    _fields_ = [("tail", ctypes.c_uint64), ("stream_hash", ctypes.c_uint64), ("token", ctypes.c_uint32),
                ("_pad", ctypes.c_uint32)]


class c_opts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("_pad", ctypes.c_uint32), ("max_configs", ctypes.c_uint64), ("stream", ctypes.c_void_p),
                ("timeout_us", ctypes.c_uint64), ("engine", ctypes.c_uint32), ("reductions_off", ctypes.c_uint32),
                ("devices", ctypes.POINTER(ctypes.c_int32)), ("n_devices", ctypes.c_uint32),
                ("_pad2", ctypes.c_uint32)]


class c_result(ctypes.Structure):
    _fields_ = [("verdict", ctypes.c_int32), ("reason", ctypes.c_int32), ("configs_explored", ctypes.c_uint64),
                ("rounds", ctypes.c_uint32), ("n_ops", ctypes.c_uint32), ("witness_len", ctypes.c_uint32),
                ("_pad", ctypes.c_uint32), ("witness", ctypes.POINTER(ctypes.c_int64)),
                ("device_ms", ctypes.c_double), ("partial", ctypes.POINTER(ctypes.c_int64)),
                ("partial_len", ctypes.c_uint32), ("_pad2", ctypes.c_uint32)]


class c_history_info(ctypes.Structure):
    _fields_ = [("n_events", ctypes.c_uint32), ("n_ops", ctypes.c_uint32), ("n_chains", ctypes.c_uint32),
                ("n_tokens", ctypes.c_uint32), ("n_record_hashes", ctypes.c_uint64),
                ("structural", ctypes.c_int32), ("n_identity_ops", ctypes.c_uint32)]


class c_batch_stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("configs_explored", ctypes.c_uint64), ("children_generated", ctypes.c_uint64),
                ("rounds", ctypes.c_uint64), ("algo_bytes", ctypes.c_uint64),
                ("n_overflow", ctypes.c_uint32), ("launches", ctypes.c_uint32),
                ("level_ms", ctypes.c_double), ("level_histories", ctypes.c_uint32),
                ("level_max_frontier", ctypes.c_uint32), ("level_rounds", ctypes.c_uint64),
                ("level_configs", ctypes.c_uint64), ("level_children", ctypes.c_uint64),
                ("pack16_ms", ctypes.c_double), ("pack16_algo_bytes", ctypes.c_uint64),
                ("pack16_histories", ctypes.c_uint32), ("pack16_small", ctypes.c_uint32),
                ("level_persist_rounds", ctypes.c_uint64), ("level_persist_launches", ctypes.c_uint32),
                ("level_chunk_retries", ctypes.c_uint32), ("level_syncs", ctypes.c_uint32), ("level_solo_rounds", ctypes.c_uint32),
                ("n_ops_total", ctypes.c_uint64), ("pack8_ms", ctypes.c_double),
                ("pack8_algo_bytes", ctypes.c_uint64), ("pack8_histories", ctypes.c_uint32), ("_pad3", ctypes.c_uint32),
                ("level_persist_fallbacks", ctypes.c_uint32), ("_pad4", ctypes.c_uint32),
                ("level_narrow_ms", ctypes.c_double), ("level_wide_ms", ctypes.c_double),
                ("level_solo_ms", ctypes.c_double), ("level_grows", ctypes.c_uint32), ("_pad5", ctypes.c_uint32)]


class c_sim_params(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("workflow", ctypes.c_uint32),
                ("num_clients", ctypes.c_uint32), ("ops_per_client", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("p_indefinite", ctypes.c_double), ("p_definite", ctypes.c_double),
                ("p_read_failure", ctypes.c_double), ("p_check_tail_failure", ctypes.c_double),
                ("initial_records", ctypes.c_uint64), ("violation", ctypes.c_uint32),
                ("max_client_ids", ctypes.c_uint32)]


def _np_field(t):
    if t is ctypes.c_char_p or t is ctypes.POINTER(ctypes.c_uint64):
        return np.dtype(np.uint64)  # pointers as integers
    return np.dtype(t)


class c_partials(ctypes.Structure):
    _fields_ = [("verdict", ctypes.c_int32), ("exact", ctypes.c_uint32), ("n_ops", ctypes.c_uint32),
                ("n_partials", ctypes.c_uint32), ("op_ids", ctypes.POINTER(ctypes.c_int64)),
                ("op_partial", ctypes.POINTER(ctypes.c_uint32)), ("offs", ctypes.POINTER(ctypes.c_uint64)),
                ("ids", ctypes.POINTER(ctypes.c_int64))]


class c_dist_info(ctypes.Structure):
    _fields_ = [("config_bytes", ctypes.c_uint64), ("n_chains", ctypes.c_uint32), ("round", ctypes.c_uint32),
                ("frontier", ctypes.c_uint32), ("found_parent", ctypes.c_uint32), ("found_move", ctypes.c_uint32),
                ("found_p4", ctypes.c_uint32), ("configs", ctypes.c_uint64), ("children", ctypes.c_uint64),
                ("max_frontier", ctypes.c_uint64), ("device_ms", ctypes.c_double), ("trace_len", ctypes.c_uint64),
                ("frontier_cap", ctypes.c_uint64)]


class c_dist_xstat(ctypes.Structure):
    _fields_ = [("ran", ctypes.c_uint32), ("done", ctypes.c_uint32), ("nf", ctypes.c_uint32),
                ("maxblk", ctypes.c_uint32), ("nf_global", ctypes.c_uint64), ("staged", ctypes.c_uint64)]


# s2lc_dist_x_* stops (include/s2lincheck.h)
DIST_X_RUNNING, DIST_X_FOUND, DIST_X_EMPTY, DIST_X_CAPACITY, DIST_X_ABORT = 0, 1, 2, 4, 5


# s2lc_event as a numpy structured dtype (bulk export without Python loops)
EVENT_NP_DTYPE = np.dtype({"names": [f for f, _ in c_event._fields_],
                           "formats": [_np_field(t) for _, t in c_event._fields_],
                           "offsets": [getattr(c_event, f).offset for f, _ in c_event._fields_],
                           "itemsize": ctypes.sizeof(c_event)})


# Every symbol include/s2lincheck.h declares: (name, restype, argtypes)
_P = ctypes.c_void_p
SIGNATURES = [
    ("s2lc_create", _P, [ctypes.POINTER(c_opts), ctypes.POINTER(ctypes.c_int)]),
    ("s2lc_destroy", None, [_P]),
    ("s2lc_last_error", ctypes.c_char_p, [_P]),
    ("s2lc_version", ctypes.c_char_p, []),
    ("s2lc_load_jsonl", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_P),
                                       ctypes.c_char_p, ctypes.c_size_t]),
    ("s2lc_history_from_events", ctypes.c_int, [ctypes.POINTER(c_event), ctypes.c_size_t, ctypes.POINTER(_P),
                                                ctypes.c_char_p, ctypes.c_size_t]),
    ("s2lc_history_free", None, [_P]),
    ("s2lc_history_pool_trim", ctypes.c_size_t, []),
    ("s2lc_history_event_count", ctypes.c_size_t, [_P]),
    ("s2lc_history_get_event", ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(c_event)]),
    ("s2lc_history_get_events", ctypes.c_int, [_P, _P, ctypes.c_size_t]),
    ("s2lc_history_info_get", ctypes.c_int, [_P, ctypes.POINTER(c_history_info)]),
    ("s2lc_check", ctypes.c_int, [_P, _P, ctypes.POINTER(c_result)]),
    ("s2lc_check_batch", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.c_size_t, ctypes.POINTER(c_result)]),
    ("s2lc_result_free", None, [ctypes.POINTER(c_result)]),
    ("s2lc_batch_create", ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.c_size_t, ctypes.POINTER(_P)]),
    ("s2lc_batch_check", ctypes.c_int, [_P, _P, ctypes.POINTER(c_result)]),
    ("s2lc_batch_load", ctypes.c_int, [_P, _P, ctypes.POINTER(_P), ctypes.c_size_t]),
    ("s2lc_batch_run", ctypes.c_int, [_P, _P]),
    ("s2lc_batch_results", ctypes.c_int, [_P, _P, ctypes.POINTER(c_result), ctypes.c_int]),
    ("s2lc_batch_results_flat", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    ("s2lc_batch_free", None, [_P]),
    ("s2lc_batch_stats_get", ctypes.c_int, [_P, ctypes.POINTER(c_batch_stats)]),
    ("s2lc_batch_run_totals", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    ("s2lc_batch_round_counts", ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t,
                                               ctypes.POINTER(ctypes.c_size_t)]),
    ("s2lc_device_fold", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_uint64)]),
    ("s2lc_step_cpu", ctypes.c_int, [_P, ctypes.POINTER(c_state), ctypes.c_uint32, ctypes.POINTER(c_state)]),
    ("s2lc_chain_hash", ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    ("s2lc_fold_record_hashes", ctypes.c_uint64, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]),
    ("s2lc_replay", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]),
    ("s2lc_sim_params_default", None, [ctypes.POINTER(c_sim_params)]),
    ("s2lc_simulate_jsonl", ctypes.c_int, [ctypes.POINTER(c_sim_params), ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                           ctypes.POINTER(ctypes.c_size_t)]),
    ("s2lc_simulate_history", ctypes.c_int, [ctypes.POINTER(c_sim_params), ctypes.POINTER(_P)]),
    ("s2lc_free", None, [_P]),
    ("s2lc_load_jsonl_many", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_P),
                                            ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]),
    ("s2lc_visualize", ctypes.c_int, [_P, ctypes.POINTER(c_result), ctypes.c_char_p]),
    ("s2lc_describe_operation", ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]),
    ("s2lc_describe_state", ctypes.c_int, [_P, ctypes.POINTER(c_state), ctypes.c_char_p, ctypes.c_size_t]),
    ("s2lc_check_partials", ctypes.c_int, [_P, _P, ctypes.POINTER(c_partials)]),
    ("s2lc_visualize_info", ctypes.c_int, [_P, ctypes.POINTER(c_result), ctypes.POINTER(c_partials), ctypes.c_char_p]),
    ("s2lc_partials_free", None, [ctypes.POINTER(c_partials)]),
    ("s2lc_history_save_many", ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                              ctypes.POINTER(ctypes.c_size_t)]),
    ("s2lc_history_load_many", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_P),
                                              ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    ("s2lc_witness_from_moves", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int64), ctypes.c_size_t]),
    ("s2lc_dist_create", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]),
    ("s2lc_dist_free", None, [_P]),
    ("s2lc_dist_expand", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int32)]),
    ("s2lc_dist_pack", ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_uint64)]),
    ("s2lc_dist_insert", ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("s2lc_dist_info", ctypes.c_int, [_P, ctypes.POINTER(c_dist_info)]),
    ("s2lc_dist_trace", ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("s2lc_dist_local_round", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int32)]),
    ("s2lc_dist_local_run", ctypes.c_int, [_P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint32)]),
    ("s2lc_dist_keep_owned", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("s2lc_dist_frontier_pack", ctypes.c_int, [_P, _P]),
    ("s2lc_dist_frontier_load", ctypes.c_int, [_P, _P, ctypes.c_uint64]),
    ("s2lc_dist_x_begin", ctypes.c_int, [_P]),
    ("s2lc_dist_x_send", ctypes.c_int, [_P, _P, ctypes.c_uint32]),
    ("s2lc_dist_x_recv", ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    ("s2lc_dist_x_wait", ctypes.c_int, [_P, ctypes.c_uint32, ctypes.POINTER(c_dist_xstat)]),
    ("s2lc_dist_x_rewind", ctypes.c_int, [_P, ctypes.c_uint32]),
    ("s2lc_dist_x_end", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)]),
]

_lib = None


def lib():
    """Load libs2lincheck.so (built in-tree by `make -C s2_verification_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `make -C s2_verification_amd` "
                              "(or __graft_entry__.build()); there is no fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# -------------------------------------------------------------- the model ---
def chain_hash(stream_hash: int, record_hash: int) -> int:
    """chainHash, main.go:232-236."""
    return lib().s2lc_chain_hash(stream_hash, record_hash)


def fold_record_hashes(stream_hash: int, record_hashes: Sequence[int]) -> int:
    """foldRecordHashes, main.go:238-244."""
    arr = (ctypes.c_uint64 * len(record_hashes))(*record_hashes)
    return lib().s2lc_fold_record_hashes(stream_hash, arr, len(record_hashes))


def Ptr(v):  # main.go:525 — pointers are plain Optional values here
    return v


@dataclass
class StreamInput:
    """main.go:206-215. 0 append, 1 read, 2 check-tail."""
    InputType: int = 0
    SetFencingToken: Optional[str] = None
    BatchFencingToken: Optional[str] = None
    MatchSeqNum: Optional[int] = None
    NumRecords: Optional[int] = None
    RecordHashes: List[int] = field(default_factory=list)


@dataclass
class StreamOutput:
    """main.go:217-225."""
    Failure: bool = False
    DefiniteFailure: bool = False
    Tail: Optional[int] = None
    StreamHash: Optional[int] = None


@dataclass
class Event:
    """porcupine.Event."""
    Kind: int
    Value: object
    Id: int
    ClientId: int = 0


def _to_c_events(events: Sequence[Event]):
    arr = (c_event * len(events))()
    keep = []
    for i, e in enumerate(events):
        c = arr[i]
        c.kind = e.Kind
        c.op_id = e.Id
        c.client_id = e.ClientId
        v = e.Value
        if e.Kind == CallEvent:
            c.input_type = v.InputType
            c.has_num_records = v.NumRecords is not None
            c.num_records = v.NumRecords or 0
            c.has_match_seq_num = v.MatchSeqNum is not None
            c.match_seq_num = v.MatchSeqNum or 0
            if v.SetFencingToken is not None:
                b = v.SetFencingToken.encode()
                keep.append(b)
                c.set_fencing_token = b
            if v.BatchFencingToken is not None:
                b = v.BatchFencingToken.encode()
                keep.append(b)
                c.fencing_token = b
            hs = list(v.RecordHashes or [])
            if hs:
                h = (ctypes.c_uint64 * len(hs))(*hs)
                keep.append(h)
                c.record_hashes = h
            c.n_record_hashes = len(hs)
        else:
            c.failure = bool(v.Failure)
            c.definite_failure = bool(v.DefiniteFailure)
            c.has_tail = v.Tail is not None
            c.tail = v.Tail or 0
            c.has_stream_hash = v.StreamHash is not None
            c.stream_hash = v.StreamHash or 0
    return arr, keep


class History:
    """An s2lc_history: decoded events + the device search layout."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.s2lc_history_free(h)

    @classmethod
    def from_events(cls, events: Sequence[Event]) -> "History":
        arr, keep = _to_c_events(events)
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        rc = lib().s2lc_history_from_events(arr, len(events), ctypes.byref(out), err, 1024)
        if rc:
            raise S2LCError(rc, err.value.decode(errors="replace"))
        return cls(out.value)

    @classmethod
    def from_jsonl(cls, data=None, path=None) -> "History":
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(2048)
        if data is not None:
            if isinstance(data, str):
                data = data.encode()
            rc = lib().s2lc_load_jsonl(None, data, len(data), ctypes.byref(out), err, 2048)
        else:
            rc = lib().s2lc_load_jsonl(path.encode(), None, 0, ctypes.byref(out), err, 2048)
        if rc:
            raise S2LCError(rc, err.value.decode(errors="replace"))
        return cls(out.value)

    def info(self) -> dict:
        i = c_history_info()
        lib().s2lc_history_info_get(self._h, ctypes.byref(i))
        return {k: getattr(i, k) for k, _ in c_history_info._fields_}

    def __len__(self):
        return lib().s2lc_history_event_count(self._h)

    def events(self) -> List[Event]:
        out = []
        e = c_event()
        for i in range(len(self)):
            lib().s2lc_history_get_event(self._h, i, ctypes.byref(e))
            if e.kind == CallEvent:
                hs = [e.record_hashes[k] for k in range(e.n_record_hashes)] if e.n_record_hashes else []
                v = StreamInput(InputType=e.input_type,
                                SetFencingToken=e.set_fencing_token.decode() if e.set_fencing_token else None,
                                BatchFencingToken=e.fencing_token.decode() if e.fencing_token else None,
                                MatchSeqNum=e.match_seq_num if e.has_match_seq_num else None,
                                NumRecords=e.num_records if e.has_num_records else None,
                                RecordHashes=hs)
            else:
                v = StreamOutput(Failure=bool(e.failure), DefiniteFailure=bool(e.definite_failure),
                                 Tail=e.tail if e.has_tail else None,
                                 StreamHash=e.stream_hash if e.has_stream_hash else None)
            out.append(Event(e.kind, v, e.op_id, e.client_id))
        return out

    def events_numpy(self):
        """All events as a numpy structured array in the s2lc_event layout (zero Python loops)."""
        n = len(self)
        arr = np.zeros(n, dtype=EVENT_NP_DTYPE)
        rc = lib().s2lc_history_get_events(self._h, arr.ctypes.data, n)
        if rc:
            raise S2LCError(rc, "get_events")
        return arr

    def step(self, state: Tuple[int, int, int], op_index: int):
        """s2Model.Step for dense op `op_index` from (tail, hash, token_id)."""
        s = c_state(state[0], state[1], state[2], 0)
        outs = (c_state * 2)()
        n = lib().s2lc_step_cpu(self._h, ctypes.byref(s), op_index, outs)
        if n < 0:
            raise S2LCError(n, "step")
        return [(outs[k].tail, outs[k].stream_hash, outs[k].token) for k in range(n)]

    def describe_operation(self, op_index: int) -> str:
        """s2Model.DescribeOperation (main.go:341-352) of dense op `op_index`."""
        n = lib().s2lc_describe_operation(self._h, op_index, None, 0)
        if n < 0:
            raise S2LCError(n, "describe_operation")
        buf = ctypes.create_string_buffer(n + 1)
        lib().s2lc_describe_operation(self._h, op_index, buf, n + 1)
        return buf.value.decode()

    def describe_state(self, state: Tuple[int, int, int]) -> str:
        """s2Model.DescribeState (main.go:353-360) of (tail, hash, token_id)."""
        s = c_state(state[0], state[1], state[2], 0)
        n = lib().s2lc_describe_state(self._h, ctypes.byref(s), None, 0)
        if n < 0:
            raise S2LCError(n, "describe_state")
        buf = ctypes.create_string_buffer(n + 1)
        lib().s2lc_describe_state(self._h, ctypes.byref(s), buf, n + 1)
        return buf.value.decode()

    def replay(self, order: Sequence[int]) -> bool:
        arr = (ctypes.c_uint32 * len(order))(*order)
        return lib().s2lc_replay(self._h, arr, len(order)) == 0


def load_many(blobs: Sequence[bytes], threads: int = 0) -> List[History]:
    """Decode many JSONL histories in parallel (s2lc_load_jsonl_many)."""
    n = len(blobs)
    # one c_char_p array over the bytes objects (it points into them, no copy,
    # and holds them); lengths and handles as numpy arrays. (Per-blob ctypes
    # objects cost ~3 us each: 30 ms for a 10k batch, half the decode.)
    keep = [b if type(b) is bytes else bytes(b) for b in blobs]
    arr = (ctypes.c_char_p * max(1, n))(*keep)
    bufs = ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p))
    lens = np.fromiter(map(len, keep), np.uint64, n) if n else np.zeros(1, np.uint64)
    out = np.zeros(max(1, n), np.uint64)
    bad = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(1024)
    rc = lib().s2lc_load_jsonl_many(bufs, lens.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)), n, threads,
                                    out.ctypes.data_as(ctypes.POINTER(_P)), ctypes.byref(bad), err, 1024)
    if rc:
        raise S2LCError(rc, err.value.decode(errors="replace"))
    return list(map(History, out[:n].tolist()))


def save_cache(hs: Sequence[History]) -> bytes:
    """s2lc_history_save_many: the binary SoA cache image of `hs` (decoded and
    finalized; load_cache skips JSONL decode)."""
    arr = (ctypes.c_void_p * max(1, len(hs)))(*[h._h for h in hs])
    buf = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    rc = lib().s2lc_history_save_many(arr, len(hs), ctypes.byref(buf), ctypes.byref(n))
    if rc:
        raise S2LCError(rc, "save_cache")
    data = ctypes.string_at(buf, n.value)
    lib().s2lc_free(buf)
    return data


def history_pool_trim() -> int:
    """s2lc_history_pool_trim: return the released histories the decoders keep
    for reuse (S2LC_HISTORY_POOL_MB) to the C heap; the array bytes released."""
    return int(lib().s2lc_history_pool_trim())


def load_cache(data: bytes, threads: int = 0) -> List[History]:
    """s2lc_history_load_many: histories from a save_cache image (bytes, or a
    read-only buffer such as an mmap of a cache file)."""
    if not isinstance(data, bytes):
        data = bytes(data)
    n = ctypes.c_size_t()
    rc = lib().s2lc_history_load_many(data, len(data), threads, None, 0, ctypes.byref(n))
    if rc:
        raise S2LCError(rc, "load_cache: not a history cache image")
    out = np.zeros(max(1, n.value), np.uint64)
    rc = lib().s2lc_history_load_many(data, len(data), threads, out.ctypes.data_as(ctypes.POINTER(_P)), n.value,
                                      ctypes.byref(n))
    if rc:
        raise S2LCError(rc, "load_cache: malformed history cache image")
    return list(map(History, out[:n.value].tolist()))


def events_from_reader(data) -> History:
    """eventsFromReader (main.go:529-563): bytes/str JSONL -> History (raises on decode error)."""
    return History.from_jsonl(data=data)


def load_file(path: str) -> History:
    return History.from_jsonl(path=path)


@dataclass
class LinearizationInfo:
    """porcupine.LinearizationInfo for one partition (S2 has one): the distinct
    partial linearizations (lists of Event.Id) and, per Event.Id, the index of
    the longest one containing it (None: in none)."""
    verdict: str
    exact: bool
    partial_linearizations: List[List[int]]
    largest: dict


@dataclass
class CheckResult:
    verdict: str
    reason: str
    configs_explored: int
    rounds: int
    n_ops: int
    witness: Optional[List[int]]
    device_ms: float
    partial: Optional[List[int]] = None  # Illegal: deepest certified linearized prefix (Event.Ids)


def _ids(ptr, n, as_numpy):
    if not ptr:
        return None
    a = np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0, dtype=np.int64)
    return a if as_numpy else a.tolist()


def _convert(r: c_result, as_numpy: bool = False) -> CheckResult:
    """c_result -> CheckResult; witness / partial as lists of Event.Ids (numpy
    int64 arrays with as_numpy, a memcpy instead of one Python int per op)."""
    return CheckResult(_VERDICT[r.verdict], REASONS.get(r.reason, str(r.reason)), r.configs_explored,
                       r.rounds, r.n_ops, _ids(r.witness, r.witness_len, as_numpy), r.device_ms,
                       _ids(r.partial, r.partial_len, as_numpy))


class Batch:
    """Device-resident batch of histories (upload once, check repeatedly)."""

    def __init__(self, checker: "Checker", histories: Sequence[History]):
        self.checker = checker
        self.histories = list(histories)
        arr = (ctypes.c_void_p * len(self.histories))(*[h._h for h in self.histories])
        out = ctypes.c_void_p()
        rc = lib().s2lc_batch_create(checker._ctx, arr, len(self.histories), ctypes.byref(out))
        if rc:
            raise S2LCError(rc, checker.last_error())
        self._b = out.value

    def __del__(self):
        b, self._b = getattr(self, "_b", None), None
        if b and _lib is not None:
            _lib.s2lc_batch_free(b)

    def load(self, histories: Sequence[History]):
        """s2lc_batch_load: replace the histories, reusing the device buffers."""
        hs = list(histories)
        arr = np.fromiter((h._h or 0 for h in hs), np.uint64, len(hs)) if hs else np.zeros(1, np.uint64)
        rc = lib().s2lc_batch_load(self.checker._ctx, self._b, arr.ctypes.data_as(ctypes.POINTER(_P)), len(hs))
        if rc:
            raise S2LCError(rc, self.checker.last_error())
        self.histories = hs
        self._detached = False

    def _check_attached(self):
        # (check_jsonl_many releases a pipe batch's histories once certified:
        # its device results then have no host histories to refer to)
        if getattr(self, "_detached", False):
            raise RuntimeError("the batch's histories were released; load() new histories first")

    def run(self):
        self._check_attached()
        rc = lib().s2lc_batch_run(self.checker._ctx, self._b)
        if rc:
            raise S2LCError(rc, self.checker.last_error())

    def results(self, with_witness=True, as_numpy=False) -> List[CheckResult]:
        self._check_attached()
        n = len(self.histories)
        res = (c_result * max(n, 1))()
        rc = lib().s2lc_batch_results(self.checker._ctx, self._b, res, int(with_witness))
        out = [_convert(res[i], as_numpy) for i in range(n)] if rc in (0, EWITNESS) else None
        for i in range(n):
            lib().s2lc_result_free(ctypes.byref(res[i]))
        if rc:
            raise S2LCError(rc, self.checker.last_error())
        return out

    def results_flat(self, with_witness=True) -> dict:
        """s2lc_batch_results_flat: numpy arrays (verdict, reason, configs,
        rounds per history; certified Ok witnesses as one int64 array of op ids
        with offsets: history i's witness = witness_ids[offs[i]:offs[i+1]])."""
        self._check_attached()
        n = len(self.histories)
        out = {"verdict": np.zeros(n, np.int32), "reason": np.zeros(n, np.int32),
               "configs": np.zeros(n, np.uint64), "rounds": np.zeros(n, np.uint64),
               "witness_offs": np.zeros(n + 1, np.uint64)}
        cap = self.stats()["n_ops_total"] if with_witness else 0
        ids = np.zeros(max(1, cap), np.int64)
        p = lambda a: a.ctypes.data
        rc = lib().s2lc_batch_results_flat(self.checker._ctx, self._b, p(out["verdict"]), p(out["reason"]),
                                           p(out["configs"]), p(out["rounds"]), p(ids) if with_witness else None,
                                           cap, p(out["witness_offs"]))
        if rc and rc != EWITNESS:
            raise S2LCError(rc, self.checker.last_error())
        out["witness_ids"] = ids[:int(out["witness_offs"][-1])]
        if rc:
            raise S2LCError(rc, self.checker.last_error())
        return out

    def round_counts(self, i: int) -> List[int]:
        """Unique configurations of each completed round of history i's last
        search (the checker needs round_counts=True)."""
        n = ctypes.c_size_t(0)
        rc = lib().s2lc_batch_round_counts(self._b, i, None, 0, ctypes.byref(n))
        if rc:
            raise S2LCError(rc, "round counts (Checker(round_counts=True) and a run first)")
        buf = (ctypes.c_uint32 * max(1, n.value))()
        rc = lib().s2lc_batch_round_counts(self._b, i, buf, n.value, ctypes.byref(n))
        if rc:
            raise S2LCError(rc, "round counts")
        return list(buf[:n.value])

    def check(self, with_witness=True) -> List[CheckResult]:
        self.run()
        return self.results(with_witness)

    def stats(self) -> dict:
        s = c_batch_stats()
        lib().s2lc_batch_stats_get(self._b, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in c_batch_stats._fields_}

    def run_totals(self) -> dict:
        """s2lc_batch_run_totals: runs so far and the sums of their kernel /
        pack_kernel<16> / pack_kernel<8> milliseconds."""
        n = ctypes.c_uint64()
        k, p16, p8 = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        lib().s2lc_batch_run_totals(self._b, ctypes.byref(n), ctypes.byref(k), ctypes.byref(p16), ctypes.byref(p8))
        return {"runs": n.value, "kernel_ms": k.value, "pack16_ms": p16.value, "pack8_ms": p8.value}


class Checker:
    """An s2lc_ctx bound to one HIP device (and optionally an existing stream).

    timeout: seconds, porcupine's CheckEventsVerbose timeout (0 = none).
    engine: ENGINE_* to force a search engine; reductions_off: RED_* bits;
    round_counts: record per-round configuration counts (Batch.round_counts);
    devices: HIP ordinals for check_batch sharding (LPT placement)."""

    def __init__(self, device: int = -1, witness: bool = True, max_configs: int = 0, stream: int = 0,
                 timeout: float = 0, engine: int = ENGINE_AUTO, reductions_off: int = 0,
                 round_counts: bool = False, devices: Optional[Sequence[int]] = None):
        o = c_opts()
        o.struct_size = ctypes.sizeof(c_opts)
        o.device = device
        o.flags = (0 if witness else F_NO_WITNESS) | (F_ROUND_COUNTS if round_counts else 0)
        o.max_configs = max_configs
        o.stream = stream or None
        o.timeout_us = int(round(timeout * 1e6)) if timeout else 0
        o.engine = engine
        o.reductions_off = reductions_off
        if devices:
            self._devs = (ctypes.c_int32 * len(devices))(*devices)
            o.devices = self._devs
            o.n_devices = len(devices)
        st = ctypes.c_int(0)
        ctx = lib().s2lc_create(ctypes.byref(o), ctypes.byref(st))
        if not ctx:
            raise S2LCError(st.value, "no usable HIP device for the S2 checker")
        self._ctx = ctx
        self.stream = stream or 0  # the caller's hipStream_t the context launches on (0: its own)

    def __del__(self):
        c, self._ctx = getattr(self, "_ctx", None), None
        if c and _lib is not None:
            _lib.s2lc_destroy(c)

    def last_error(self) -> str:
        return lib().s2lc_last_error(self._ctx).decode(errors="replace")

    def check(self, h: History) -> CheckResult:
        """s2lc_check: one history through the context's reusable scratch batch."""
        r = c_result()
        rc = lib().s2lc_check(self._ctx, h._h, ctypes.byref(r))
        out = _convert(r) if rc in (0, EWITNESS) else None
        lib().s2lc_result_free(ctypes.byref(r))
        if rc:
            raise S2LCError(rc, self.last_error())
        return out

    def check_many(self, hs: Sequence[History], as_numpy: bool = False) -> List[CheckResult]:
        """s2lc_check_batch: the context's scratch (no allocation once warm),
        sharded over the context's devices when it has several."""
        n = len(hs)
        arr = (ctypes.c_void_p * max(1, n))(*[h._h for h in hs])
        res = (c_result * max(1, n))()
        rc = lib().s2lc_check_batch(self._ctx, arr, n, res)
        out = [_convert(res[i], as_numpy) for i in range(n)] if rc in (0, EWITNESS) else None
        for i in range(n):
            lib().s2lc_result_free(ctypes.byref(res[i]))
        if rc:
            raise S2LCError(rc, self.last_error())
        return out

    def partials(self, h: History) -> "LinearizationInfo":
        """s2lc_check_partials: porcupine's LinearizationInfo for one history
        (the longest certified partial linearization containing each op)."""
        p = c_partials()
        rc = lib().s2lc_check_partials(self._ctx, h._h, ctypes.byref(p))
        if rc:
            raise S2LCError(rc, self.last_error())
        try:
            n, k = p.n_ops, p.n_partials
            offs = [p.offs[i] for i in range(k + 1)]
            parts = [[p.ids[x] for x in range(offs[i], offs[i + 1])] for i in range(k)]
            op_ids = [p.op_ids[d] for d in range(n)]
            op_part = [p.op_partial[d] for d in range(n)]
            largest = {op_ids[d]: (op_part[d] if op_part[d] != 0xFFFFFFFF else None) for d in range(n)}
            return LinearizationInfo(_VERDICT[p.verdict], bool(p.exact), parts, largest)
        finally:
            lib().s2lc_partials_free(ctypes.byref(p))

    def device_fold(self, seeds, folds):
        """foldRecordHashes on the GPU (the search kernels' device routine):
        [fold(seeds[i], folds[i]) for i]."""
        n = len(seeds)
        pool = [x for f in folds for x in f]
        offs, o = [], 0
        for f in folds:
            offs.append(o)
            o += len(f)
        sd = (ctypes.c_uint64 * max(1, n))(*seeds)
        pl = (ctypes.c_uint64 * max(1, len(pool)))(*pool)
        of = (ctypes.c_uint32 * max(1, n))(*offs)
        ct = (ctypes.c_uint32 * max(1, n))(*[len(f) for f in folds])
        out = (ctypes.c_uint64 * max(1, n))()
        rc = lib().s2lc_device_fold(self._ctx, sd, pl, len(pool), of, ct, n, out)
        if rc:
            raise S2LCError(rc, self.last_error())
        return list(out[:n])

    def check_batch(self, hs: Sequence[History]) -> List[CheckResult]:
        return Batch(self, hs).check()

    def check_jsonl_many(self, blobs: Sequence[bytes], threads: int = 0, slices: int = 2,
                         with_witness: bool = True, overlap: Optional[bool] = None) -> dict:
        """Collector JSONL blobs (one history each) -> Batch.results_flat's
        arrays, in input order, pipelined over `slices` slices of the input:
        slice k+1 decodes on the host cores while slice k uploads and runs on
        the device, and slice k's witnesses are certified while slice k+1
        uploads and runs (the copy engine and the GPU work beside the decoder
        and certifier threads). With `overlap` (default: S2LC_PIPE_OVERLAP=1)
        the certification of slice k also runs beside the decode of slice k+2
        on a thread of its own, instead of between the decodes. Two device
        batches alternate and are kept on the checker for the next call (a
        long-running checker: warm buffers).

        A context is single-threaded (include/s2lincheck.h): the device stage
        (load + run) and the certification (results_flat) of different slices
        run on different threads, so each takes the checker's lock around its
        context calls (they had shared the context's error slot and
        its stream unguarded). The decode (s2lc_load_jsonl_many) needs no
        context and runs beside either."""
        import threading
        from concurrent.futures import ThreadPoolExecutor
        n = len(blobs)
        S = max(1, min(int(slices), n))
        cuts = [n * k // S for k in range(S + 1)]
        if overlap is None:
            overlap = os.environ.get("S2LC_PIPE_OVERLAP", "0") == "1"
        if not hasattr(self, "_pipe"):
            self._pipe = [None, None]
            self._ctx_lock = threading.Lock()
        lock = self._ctx_lock

        def device(slot, hs):
            with lock:
                b = self._pipe[slot]
                if b is None:
                    b = self._pipe[slot] = Batch(self, hs)
                else:
                    b.load(hs)
                b.run()
            return b

        def certify(b):
            with lock:
                o = b.results_flat(with_witness)
            # release the slice's host histories as soon as they are certified:
            # the next slice's decode then reuses their storage (the history
            # pool) instead of faulting in fresh pages. The pipe batch is not
            # read again before its next load().
            b.histories = []
            b._detached = True
            return o

        outs = []
        with ThreadPoolExecutor(1) as ex, ThreadPoolExecutor(1) as cx:
            fut = None
            slot_cert = [None, None]  # (overlap) the pending certification of each device batch
            for k in range(S):
                hs = load_many(blobs[cuts[k]:cuts[k + 1]], threads=threads)  # (ctypes: the GIL is released)
                prev = fut.result() if fut is not None else None
                if overlap:
                    if prev is not None:
                        slot_cert[(k - 1) % 2] = cx.submit(certify, prev)
                        outs.append(slot_cert[(k - 1) % 2])
                    if slot_cert[k % 2] is not None:  # its batch held slice k-2: certified before reuse
                        slot_cert[k % 2].result()
                    fut = ex.submit(device, k % 2, hs)
                    del hs
                    continue
                fut = ex.submit(device, k % 2, hs)
                del hs
                if prev is not None:
                    outs.append(certify(prev))
            if overlap:
                outs.append(cx.submit(certify, fut.result()))
                outs = [f.result() for f in outs]
            else:
                outs.append(certify(fut.result()))
        res = {}
        for key in ("verdict", "reason", "configs", "rounds"):
            res[key] = np.concatenate([o[key] for o in outs])
        res["witness_ids"] = np.concatenate([o["witness_ids"] for o in outs])
        offs, base = [np.zeros(1, np.uint64)], 0
        for o in outs:
            offs.append(o["witness_offs"][1:] + np.uint64(base))
            base += int(o["witness_offs"][-1])
        res["witness_offs"] = np.concatenate(offs)
        return res

    def batch(self, hs: Sequence[History]) -> Batch:
        return Batch(self, hs)


_checkers = {}


def check_events_verbose(model, events, timeout: float = 0):
    """porcupine.CheckEventsVerbose(s2Model.ToModel(), events, timeout) on the GPU.

    `model` is accepted for signature parity and ignored (the S2 model is built in).
    timeout is in seconds (Go's time.Duration; 0 = none, as at main.go:606):
    past it the verdict is Unknown. Returns (verdict, info); info carries the
    witness linearization (op ids) for Ok, configs explored and rounds.
    """
    key = float(timeout or 0)
    if key not in _checkers:
        # a context holds device scratch sized from free HBM: keep the last
        # two timeouts' contexts, not one per distinct value
        while len(_checkers) >= 2:
            _checkers.pop(next(iter(_checkers)))
        _checkers[key] = Checker(timeout=key)
    h = events if isinstance(events, History) else History.from_events(events)
    r = _checkers[key].check(h)
    return r.verdict, r


s2Model = None  # the S2 model lives on the device; kept for call-site parity


# -------------------------------------------------------------- simulator ---
def sim_params(workflow=WF_REGULAR, num_clients=5, ops_per_client=100, seed=1, **kw) -> c_sim_params:
    p = c_sim_params()
    lib().s2lc_sim_params_default(ctypes.byref(p))
    p.workflow = workflow
    p.num_clients = num_clients
    p.ops_per_client = ops_per_client
    p.seed = seed
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def simulate_jsonl(**kw) -> bytes:
    p = sim_params(**kw)
    buf = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    rc = lib().s2lc_simulate_jsonl(ctypes.byref(p), ctypes.byref(buf), ctypes.byref(n))
    if rc:
        raise S2LCError(rc, "simulate")
    data = ctypes.string_at(buf, n.value)
    lib().s2lc_free(buf)
    return data


def simulate_history(**kw) -> History:
    p = sim_params(**kw)
    out = ctypes.c_void_p()
    rc = lib().s2lc_simulate_history(ctypes.byref(p), ctypes.byref(out))
    if rc:
        raise S2LCError(rc, "simulate")
    return History(out.value)
