"""Distributed search of ONE history across GPUs (BASELINE config C5).

One process per GPU. Configurations are hash-partitioned by fingerprint
(`lv_owner` in csrc/level_dev.h); each round every rank expands and closes its
own frontier on its GPU (libs2lincheck: s2lc_dist_expand / s2lc_dist_pack),
the closed children travel to their owner rank in ONE all-to-all(v) over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X), and the owner
deduplicates them in its HBM table (s2lc_dist_insert). Per round there are two
collectives: a small all-to-all of (count, found, staged total) triples, which
also carries termination (Ok anywhere / nothing staged anywhere = Illegal), and
the payload all-to-all. The gloo backend works too (payload staged through host
memory), which is how the protocol is tested with several ranks on one GPU.

This replaces porcupine.CheckEventsVerbose (golang/s2-porcupine/main.go:606)
for a single history too large for one device's search; the verdict is the
same question and the Ok witness is rebuilt from the ranks' trace pools and
certified through the CPU model (s2lc_witness_from_moves).
"""
import ctypes
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import (DIST_X_ABORT, DIST_X_CAPACITY, DIST_X_EMPTY, DIST_X_FOUND, History, Illegal, Ok, S2LCError,
               c_dist_info, c_dist_xstat, lib)

_NONE = 0xFFFFFFFF
_RANK_SHIFT = 29


@dataclass
class DistResult:
    verdict: str
    rounds: int
    configs: int             # unique configurations, all ranks
    children: int            # children generated, all ranks
    max_frontier: int        # largest per-rank frontier
    device_ms: float         # max over ranks of the kernels' device time
    wall_s: float            # the search loop (all ranks in lockstep)
    exchanged_bytes: int     # payload bytes this rank sent to other ranks
    witness: Optional[List[int]] = None
    witness_valid: Optional[bool] = None
    per_rank_configs: List[int] = field(default_factory=list)  # [partitioned rounds]
    xreruns: int = 0         # partitioned rounds re-run with larger exchange blocks
    part_s: float = 0.0      # wall time of the partitioned rounds (the switches to them included)


class DistSearch:
    """One rank's share of the search (an s2lc_dist)."""

    def __init__(self, checker, history: History, rank: int, world: int):
        self._d = ctypes.c_void_p()
        rc = lib().s2lc_dist_create(checker._ctx, history._h, rank, world, ctypes.byref(self._d))
        if rc:
            raise S2LCError(rc, checker.last_error())
        self.checker = checker
        self.rank, self.world = rank, world

    def close(self):
        if self._d:
            lib().s2lc_dist_free(self._d)
            self._d = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc:
            raise S2LCError(rc, f"{what}: {self.checker.last_error()}")

    def info(self) -> c_dist_info:
        i = c_dist_info()
        self._chk(lib().s2lc_dist_info(self._d, ctypes.byref(i)), "dist_info")
        return i

    def expand(self):
        counts = (ctypes.c_uint64 * self.world)()
        found = ctypes.c_int32(0)
        self._chk(lib().s2lc_dist_expand(self._d, counts, ctypes.byref(found)), "dist_expand")
        return list(counts), bool(found.value)

    def pack(self, send: torch.Tensor, counts):
        c = (ctypes.c_uint64 * self.world)(*counts)
        self._chk(lib().s2lc_dist_pack(self._d, ctypes.c_void_p(send.data_ptr() if send.numel() else 0), c),
                  "dist_pack")

    def insert(self, recv: torch.Tensor, n: int) -> int:
        nn = ctypes.c_uint64(0)
        self._chk(lib().s2lc_dist_insert(self._d, ctypes.c_void_p(recv.data_ptr() if n else 0), n,
                                         ctypes.byref(nn)), "dist_insert")
        return nn.value

    def local_round(self):
        nn = ctypes.c_uint64(0)
        found = ctypes.c_int32(0)
        self._chk(lib().s2lc_dist_local_round(self._d, ctypes.byref(nn), ctypes.byref(found)), "dist_local_round")
        return nn.value, bool(found.value)

    def local_run(self, wide: int):
        """Replicated rounds inside the persistent kernel until the frontier
        reaches `wide` or the search ends: (frontier, found, rounds run,
        configurations inserted), or None where the kernel is unavailable
        (then: local_round)."""
        c0 = self.info().configs
        nn = ctypes.c_uint64(0)
        found = ctypes.c_int32(0)
        nr = ctypes.c_uint32(0)
        rc = lib().s2lc_dist_local_run(self._d, min(wide, 0xFFFFFFFF), ctypes.byref(nn), ctypes.byref(found),
                                       ctypes.byref(nr))
        if rc == -6:  # S2LC_EUNSUPPORTED
            return None
        self._chk(rc, "dist_local_run")
        return nn.value, bool(found.value), nr.value, self.info().configs - c0

    def keep_owned(self) -> int:
        n = ctypes.c_uint64(0)
        self._chk(lib().s2lc_dist_keep_owned(self._d, ctypes.byref(n)), "dist_keep_owned")
        return n.value

    def frontier_pack(self, buf: torch.Tensor):
        self._chk(lib().s2lc_dist_frontier_pack(self._d, ctypes.c_void_p(buf.data_ptr())), "dist_frontier_pack")

    def frontier_load(self, buf: torch.Tensor, n: int):
        self._chk(lib().s2lc_dist_frontier_load(self._d, ctypes.c_void_p(buf.data_ptr()), n), "dist_frontier_load")

    # host-free partitioned rounds (s2lc_dist_x_*, include/s2lincheck.h)
    def x_begin(self):
        self._chk(lib().s2lc_dist_x_begin(self._d), "dist_x_begin")

    def x_send(self, send: Optional[torch.Tensor], cap: int):
        ptr = ctypes.c_void_p(send.data_ptr() if send is not None else 0)
        self._chk(lib().s2lc_dist_x_send(self._d, ptr, cap), "dist_x_send")

    def x_recv(self, recv: Optional[torch.Tensor], cap: int) -> int:
        r = ctypes.c_uint32(0)
        ptr = ctypes.c_void_p(recv.data_ptr() if recv is not None else 0)
        self._chk(lib().s2lc_dist_x_recv(self._d, ptr, cap, ctypes.byref(r)), "dist_x_recv")
        return r.value

    def x_wait(self, round_: int) -> c_dist_xstat:
        st = c_dist_xstat()
        self._chk(lib().s2lc_dist_x_wait(self._d, round_, ctypes.byref(st)), "dist_x_wait")
        return st

    def x_rewind(self, round_: int):
        self._chk(lib().s2lc_dist_x_rewind(self._d, round_), "dist_x_rewind")

    def x_end(self):
        done = ctypes.c_uint32(0)
        configs = ctypes.c_uint64(0)
        self._chk(lib().s2lc_dist_x_end(self._d, ctypes.byref(done), ctypes.byref(configs)), "dist_x_end")
        return done.value, configs.value

    def trace(self) -> np.ndarray:
        n = ctypes.c_uint64(0)
        self._chk(lib().s2lc_dist_trace(self._d, None, 0, ctypes.byref(n)), "dist_trace")
        out = np.zeros((max(1, n.value), 2), dtype=np.uint32)
        self._chk(lib().s2lc_dist_trace(self._d, ctypes.c_void_p(out.ctypes.data), n.value, ctypes.byref(n)),
                  "dist_trace")
        return out[:n.value]


class _Exchange:
    """The two collectives of a round, on CUDA tensors (nccl/RCCL) or staged
    through host memory (gloo)."""

    def __init__(self, group, device: torch.device, lib_stream: int = 0):
        self.group = group
        self.device = device
        self.on_gpu = dist.get_backend(group) == "nccl"
        self.tdev = device if self.on_gpu else torch.device("cpu")
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # the library launches on torch's current stream (Checker(stream=...)):
        # its kernels are ordered after the collectives on the device, with no
        # host synchronization in between
        self.same_stream = lib_stream != 0 and lib_stream == torch.cuda.current_stream(device).cuda_stream
        # a caller stream that is not torch's current one: the
        # collectives wait for the library's queued kernels, and the
        # library's next kernels for the collectives, as stream waits on the
        # device (the library skips its host wait on a caller's stream)
        self.lib_ext = (torch.cuda.ExternalStream(lib_stream, device=device)
                        if lib_stream != 0 and not self.same_stream and device.type == "cuda" else None)

    def _pre(self):
        """Before a collective (or a host copy) reads what the library wrote."""
        if self.lib_ext is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.lib_ext)

    def _lib_sync(self):
        """After a collective, before the library reads what it received."""
        if self.same_stream or self.device.type != "cuda":
            return
        if self.lib_ext is not None:
            self.lib_ext.wait_stream(torch.cuda.current_stream(self.device))
        else:
            torch.cuda.current_stream(self.device).synchronize()  # the library reads on its own stream

    def counts(self, counts, found: bool, staged: int, frontier: int = 0):
        """All-to-all of (count for the receiver, found, staged total, the
        sender's frontier after the previous round) rows: the round's sizes,
        its termination and the previous round's global frontier in one
        collective."""
        w = self.world
        send = torch.tensor([[c, int(found), staged, frontier] for c in counts], dtype=torch.int64, device=self.tdev)
        recv = torch.empty((w, 4), dtype=torch.int64, device=self.tdev)
        dist.all_to_all_single(recv, send, group=self.group)
        r = recv.cpu().tolist()
        return [x[0] for x in r], any(x[1] for x in r), sum(x[2] for x in r), sum(x[3] for x in r)

    def payload(self, send: torch.Tensor, in_bytes, out_bytes) -> torch.Tensor:
        total = int(sum(out_bytes))
        self._pre()
        if self.on_gpu:
            recv = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
            dist.all_to_all_single(recv[:total] if total else recv[:0], send, out_bytes, in_bytes, group=self.group)
            self._lib_sync()
            return recv
        recv_h = torch.empty(total, dtype=torch.uint8)
        dist.all_to_all_single(recv_h, send.cpu(), out_bytes, in_bytes, group=self.group)
        recv = recv_h.to(self.device) if total else torch.empty(1, dtype=torch.uint8, device=self.device)
        self._lib_sync()
        return recv

    def payload_blocks(self, send: Optional[torch.Tensor], blk: int) -> Optional[torch.Tensor]:
        """All-to-all of one fixed-capacity block of `blk` bytes to every OTHER
        rank: `send` holds the world - 1 blocks in rank order without this
        rank's (its own share never travels), and so does the result, by
        sender. The split sizes are fixed, so no size goes to the host; on
        CUDA tensors (RCCL) the collective is queued behind the library's
        kernels with no host synchronization. One rank: nothing to send."""
        if self.world == 1:
            return None
        splits = [0 if r == self.rank else blk for r in range(self.world)]
        self._pre()
        if self.on_gpu:
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, splits, splits, group=self.group)
            self._lib_sync()
            return recv
        recv_h = torch.empty(send.numel(), dtype=torch.uint8)
        dist.all_to_all_single(recv_h, send.cpu(), splits, splits, group=self.group)
        recv = recv_h.to(self.device)
        self._lib_sync()
        return recv

    # (one rank: every collective below is the identity, taken on the host
    # without a device round trip)
    def sum(self, v: int) -> int:
        if self.world == 1:
            return int(v)
        t = torch.tensor([v], dtype=torch.int64, device=self.tdev)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def gather_frontier(self, mine: torch.Tensor, n_bytes: List[int]) -> torch.Tensor:
        """All-gather of variable-size byte buffers (every rank's frontier)."""
        if self.world == 1:
            return mine  # (frontier_pack waited for the library's copy)
        self._pre()
        m = max(n_bytes)
        src = torch.zeros(max(m, 1), dtype=torch.uint8, device=self.tdev)
        if n_bytes[dist.get_rank(self.group)]:
            src[:n_bytes[dist.get_rank(self.group)]] = mine[:n_bytes[dist.get_rank(self.group)]].to(self.tdev)
        out = [torch.empty(max(m, 1), dtype=torch.uint8, device=self.tdev) for _ in range(self.world)]
        dist.all_gather(out, src, group=self.group)
        full = torch.cat([out[w][:n_bytes[w]] for w in range(self.world)]) if sum(n_bytes) else out[0][:1]
        full = full.to(self.device).contiguous()
        self._lib_sync()
        return full

    def gather_small(self, vals: List[int]) -> List[List[int]]:
        if self.world == 1:
            return [[int(v) for v in vals]]
        t = torch.tensor(vals, dtype=torch.int64, device=self.tdev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [o.cpu().tolist() for o in out]

    def gather_traces(self, tr: np.ndarray) -> List[np.ndarray]:
        if self.world == 1:
            return [tr.astype(np.uint32)]
        n = self.gather_small([len(tr)])
        m = max(x[0] for x in n)
        buf = torch.zeros((max(m, 1), 2), dtype=torch.int64, device=self.tdev)
        if len(tr):
            buf[:len(tr)] = torch.from_numpy(tr.astype(np.int64)).to(self.tdev)
        out = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(out, buf, group=self.group)
        return [o[:x[0]].cpu().numpy().astype(np.uint32) for o, x in zip(out, n)]


def _walk(traces: List[np.ndarray], parent: int, move: int) -> Optional[List[int]]:
    """Moves from the root to the completing child (trace ids cross ranks)."""
    if move == _NONE:
        return []
    moves = [move]
    idx = parent
    mask = (1 << _RANK_SHIFT) - 1
    steps = 0
    while idx != _NONE:
        r, i = idx >> _RANK_SHIFT, idx & mask
        if r >= len(traces) or i >= len(traces[r]):
            return None
        p, m = int(traces[r][i][0]), int(traces[r][i][1])
        if m != _NONE:
            moves.append(m)
        idx = p
        steps += 1
        if steps > (1 << 26):
            return None
    moves.reverse()
    return moves


def bind_stream(device=None) -> int:
    """Make a dedicated torch stream current and return its handle, for
    Checker(stream=...): the library's kernels and the RCCL collectives are
    then ordered on the device, and partitioned rounds queue with no host
    synchronization. (The default stream's handle is 0, which the C ABI reads
    as "a stream of your own": the rounds then wait on the host.)"""
    s = torch.cuda.Stream(device=device)
    torch.cuda.set_stream(s)
    return s.cuda_stream


_XDEPTH = 2      # partitioned rounds queued beyond the newest status the host has read
_XDEBUG = bool(int(__import__("os").environ.get("S2LC_XDEBUG", "0") or 0))  # (diagnostics: every round's status)
_XTIME = bool(int(__import__("os").environ.get("S2LC_XTIME", "0") or 0))    # (diagnostics: host time per step)
_XRING = 8       # the library's status ring (LV_XRING): receive buffers a re-run may read


def _xcap(n: int, limit: int) -> int:
    """Exchange block capacity for an expected largest block of n: twice it,
    a power of two (a round that needs more is re-run), within the limit."""
    c = 256
    while c < 2 * n:
        c *= 2
    return max(1, min(c, limit))


@dataclass
class _XPhase:
    stop: int = 0          # DIST_X_* of the stop (0: the frontier narrowed)
    rounds: int = 0        # rounds closed in the phase (the stopping one included)
    sent_bytes: int = 0
    reruns: int = 0        # rounds re-run with a larger block capacity
    cap: int = 0           # the last block capacity
    bufs: list = field(default_factory=list)  # receive buffers; the last holds the frontier (keep it alive)


def _partitioned_rounds(ds: "DistSearch", ex: "_Exchange", device, cb: int, world: int, wide: int,
                        cap: int) -> _XPhase:
    """Partitioned rounds with no host synchronization per round
    (s2lc_dist_x_*): each round is queued as expand + block copy, one
    equal-split all-to-all of fixed-capacity blocks, and the decision +
    insert, and the host reads round r's status (the largest block it needed,
    the global frontier, the stop) while rounds r+1 .. r+_XDEPTH are queued
    behind it. A block over its capacity inserts nothing on any rank: the
    round is re-run with twice the largest block. The phase ends at a stop or
    when the global frontier narrows below wide / 4."""
    from collections import deque
    info = ds.info()
    nb = world - 1  # exchange blocks: one per other rank
    limit = max(1, int(info.frontier_cap) // (2 * max(1, nb)))
    round0 = info.round
    ph = _XPhase(cap=min(cap, limit))
    ds.x_begin()
    if _XDEBUG:
        print(f"[x] rank {ds.rank} phase from round {round0} frontier {info.frontier} cap {ph.cap} "
              f"limit {limit}", flush=True)
    queued = deque()                 # rounds whose status is not read yet
    prev_blk = 1                     # the largest block of the previous status read
    keep = deque(maxlen=_XRING + 1)  # receive buffers a re-run may start from
    tm = [0.0] * 5 if _XTIME else None
    while True:
        if tm:
            t0 = time.perf_counter()
        send = torch.empty(nb * (ph.cap + 1) * cb, dtype=torch.uint8, device=device) if nb else None
        if _XDEBUG and send is not None:
            print(f"[x] rank {ds.rank} queue cap {ph.cap} send {send.data_ptr():#x}+{send.numel()}", flush=True)
        if tm:
            t1 = time.perf_counter()
        ds.x_send(send, ph.cap)
        if tm:
            t2 = time.perf_counter()
        recv = ex.payload_blocks(send, (ph.cap + 1) * cb)
        if tm:
            t3 = time.perf_counter()
        r = ds.x_recv(recv, ph.cap)
        if tm:
            t4 = time.perf_counter()
            for i, (a, b) in enumerate(((t0, t1), (t1, t2), (t2, t3), (t3, t4))):
                tm[i] += b - a
        if _XDEBUG and recv is not None:
            print(f"[x] rank {ds.rank} queued round {r} recv {recv.data_ptr():#x}+{recv.numel()}", flush=True)
        queued.append(r)
        keep.append(recv)
        ph.sent_bytes += nb * (ph.cap + 1) * cb
        if len(queued) <= _XDEPTH:
            continue
        r0 = queued.popleft()
        if tm:
            t5 = time.perf_counter()
        st = ds.x_wait(r0)
        if tm:
            tm[4] += time.perf_counter() - t5
        if _XDEBUG:
            print(f"[x] rank {ds.rank} round {r0} cap {ph.cap} ran {st.ran} done {st.done} nf {st.nf} "
                  f"maxblk {st.maxblk} nf_global {st.nf_global} staged {st.staged}", flush=True)
        if st.done == DIST_X_CAPACITY:
            if st.maxblk > limit:
                ds.x_end()
                raise S2LCError(-5, f"distributed round {r0}: an exchange block of {st.maxblk} configurations "
                                    f"exceeds the frontier capacity ({limit} per rank)")
            ds.x_rewind(r0)
            queued.clear()
            ph.reruns += 1
            ph.cap = _xcap(st.maxblk, limit)
            continue
        if st.done:
            break
        # the status is _XDEPTH rounds old: extrapolate one step of its growth
        grow = min(8.0, max(1.0, st.maxblk / max(1, prev_blk)))
        prev_blk = st.maxblk
        ph.cap = _xcap(int(st.maxblk * grow), limit)
        if wide > 0 and r0 > round0 + 1 and st.nf_global < wide // 4:
            # narrow again. The rounds still queued run to the end of the
            # phase; one of them may stop the search or outgrow its blocks
            # (then the phase ends before it: the switch reads the frontier
            # it started from)
            for r in queued:
                st = ds.x_wait(r)
                if st.done == DIST_X_CAPACITY:
                    ds.x_rewind(r)
                    break
                if st.done:
                    break
            break
    ph.stop, _ = ds.x_end()
    if tm:
        print(f"[x] rank {ds.rank} phase host time (ms): alloc {tm[0]*1e3:.2f} send {tm[1]*1e3:.2f} "
              f"exchange {tm[2]*1e3:.2f} recv {tm[3]*1e3:.2f} wait {tm[4]*1e3:.2f} "
              f"over {ds.info().round - round0} rounds", flush=True)
    if ph.stop == DIST_X_ABORT:
        raise S2LCError(-5, "distributed round exceeds the device buffers")
    ph.rounds = ds.info().round - round0
    ph.bufs = list(keep)  # (the library's frontier is the last one queued)
    return ph


# Cost model of a partitioned round ("N-GPU model"; constants
# measured on one MI355X, profiles/r05/dist/): a round of a frontier of nf
# configurations costs the single-GPU engine ~X_FIX + X_PER * nf us; split
# over N ranks it costs X_OVER (the partitioned round's own overhead on one
# GPU) + X_RCCL (the all-to-all's latency over xGMI: a parameter, not
# measurable on one GPU) + that work / N. Partitioning pays from the frontier
# where the saving (1 - 1/N) of the work exceeds the overhead.
X_FIX, X_PER, X_OVER, X_RCCL = 10.0, 0.0082, 22.0, 30.0


def default_wide(world: int) -> int:
    """The frontier width from which rounds run partitioned on `world` ranks
    (a power of two, 4,096 .. 65,536; one rank: 4,096, the rehearsal's)."""
    if world <= 1:
        return 4096
    nf = ((X_OVER + X_RCCL) / (1.0 - 1.0 / world) - X_FIX) / X_PER
    w = 4096
    while w < nf and w < 65536:
        w *= 2
    return w


def check_distributed(checker, history: History, group=None, witness: bool = True,
                      wide: Optional[int] = None, persistent: Optional[bool] = None,
                      self_exchange: bool = False, sized_exchange: bool = False,
                      xcap0: Optional[int] = None) -> DistResult:
    """Check one history with every rank of `group` (default: the world).

    Rounds whose frontier is narrower than `wide` configurations run
    replicated (every rank the whole round, no exchange): after round 0 they
    run inside the persistent kernel of the single-GPU level search
    (s2lc_dist_local_run: solo and persistent rounds, one host sync per
    launch) unless persistent=False (one host-driven round per call). Wider
    rounds run partitioned by owner with one all-to-all per round. wide=0
    partitions every round; None: default_wide(world), from the cost model.

    persistent=None: on with nccl (one process per GPU) and for one rank; off
    for several gloo ranks, which are the tests' ranks sharing one GPU: the
    persistent grid of one process needs a workgroup resident on every CU at
    once, and kernels of other processes on the same GPU do not leave room
    for it. persistent=True there still gives the right answer: a refused
    cooperative launch or a timed-out grid barrier sends the search back to
    host-driven replicated rounds from the frontier it started from.

    self_exchange: with one rank, still switch to partitioned rounds at
    `wide` (every child goes through the all-to-all to rank 0 itself): the
    multi-GPU round sequence, rehearsed on one GPU.

    Partitioned rounds run host-free (_partitioned_rounds: fixed-capacity
    blocks, device-side decisions, no host synchronization per round);
    sized_exchange=True runs them the round-3 way instead (host-read counts,
    a variable-split all-to-all, three host synchronizations per round), kept
    for measurement. xcap0: the first exchange block capacity of each
    partitioned phase (default: from the frontier at the switch; a smaller one
    is grown by re-running the rounds that overflow it)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if wide is None:
        wide = default_wide(world)
    device = torch.device("cuda", torch.cuda.current_device())
    ex = _Exchange(group, device, getattr(checker, "stream", 0))
    if persistent is None:
        persistent = ex.on_gpu or world == 1
    ds = DistSearch(checker, history, rank, world)
    cb = ds.info().config_bytes
    keep = []  # device buffers holding this rank's frontier (kept alive)
    verdict = None
    sent_bytes = 0
    found = False
    rounds = 0
    configs = 0
    part_rounds = 0
    phase_rounds = 0  # partitioned rounds since the last switch to them
    nn_local = 0      # this rank's frontier after the last partitioned round (reported with the next counts)
    replicated = wide > 0  # wide = 0: every round partitioned (also on one rank: a self-exchange)
    nn_switch = 1          # the frontier at the switch to partitioned rounds (sizes the first exchange blocks)
    xreruns = 0            # partitioned rounds re-run with larger exchange blocks
    part_s = 0.0
    t0 = time.perf_counter()
    first = True  # round 0 closes the initial configuration; rounds counts the ones after it
    try:
        while verdict is None:
            if not first:
                rounds += 1
            first = False
            if replicated:
                split = world > 1 or self_exchange  # partitioned rounds at `wide`
                run = ds.local_run(wide if split else 1 << 32) if (persistent and rounds > 0) else None
                if run is not None:
                    nn, found, nr, dconf = run
                    rounds += nr - 1  # (this iteration counted one)
                else:
                    nn, found = ds.local_round()
                    dconf = 0 if found else nn
                configs += dconf
                if found:
                    verdict = Ok
                    break
                if nn == 0:
                    verdict = Illegal
                    break
                if split and nn >= wide:
                    ds.keep_owned()
                    nn_switch = nn
                    replicated = False
                continue
            if not sized_exchange and ds.info().round == 0:
                # (wide = 0) round 0 closes the initial configuration on every
                # rank; partitioned rounds start from it
                nn, found = ds.local_round()
                if found:
                    verdict = Ok
                    break
                if nn == 0:
                    verdict = Illegal
                    break
                configs += nn
                ds.keep_owned()
                nn_switch = nn
                continue
            if not sized_exchange:
                tp = time.perf_counter()
                c0 = ds.info().configs
                cap0 = xcap0 if xcap0 else _xcap(max(1024, 4 * nn_switch // world), 1 << 31)
                ph = _partitioned_rounds(ds, ex, device, cb, world, wide, cap0)
                keep = ph.bufs  # the frontier lives in the last one until frontier_load replaces it
                xreruns += ph.reruns
                rounds += ph.rounds - 1  # (this iteration counted one)
                part_rounds += ph.rounds
                sent_bytes += ph.sent_bytes
                configs += ex.sum(ds.info().configs - c0)
                part_s += time.perf_counter() - tp
                if ph.stop == DIST_X_FOUND:
                    found = True
                    verdict = Ok
                    break
                if ph.stop == DIST_X_EMPTY:
                    verdict = Illegal
                    break
                # narrow again: every rank takes the whole frontier
                nn = ds.info().frontier
                sizes_n = [x[0] for x in ex.gather_small([nn])]
                total = sum(sizes_n)
                mine = torch.empty(max(1, nn * cb), dtype=torch.uint8, device=device)
                if nn:
                    ds.frontier_pack(mine)
                full = ex.gather_frontier(mine, [x * cb for x in sizes_n])
                ds.frontier_load(full, total)
                keep = [full]
                replicated = True
                if total == 0:
                    verdict = Illegal
                    break
                continue
            tp = time.perf_counter()
            counts, found = ds.expand()
            # (the previous round's global frontier travels with this round's
            # counts: no collective of its own; an empty frontier shows up here
            # as nothing staged anywhere)
            recv_counts, found_any, staged_total, prev_total = ex.counts(counts, found, sum(counts), nn_local)
            if phase_rounds:
                configs += prev_total
            if found_any:
                verdict = Ok
                break
            if staged_total == 0:
                verdict = Illegal
                break
            send = torch.empty(max(1, sum(counts) * cb), dtype=torch.uint8, device=device)
            ds.pack(send, counts)
            in_b = [c * cb for c in counts]
            out_b = [c * cb for c in recv_counts]
            sent_bytes += sum(b for w, b in enumerate(in_b) if w != rank)
            recv = ex.payload(send[:sum(in_b)], in_b, out_b)
            nn = ds.insert(recv, sum(recv_counts))
            nn_local = nn
            keep = [recv]
            part_rounds += 1
            phase_rounds += 1
            part_s += time.perf_counter() - tp
            if wide > 0 and phase_rounds > 1 and prev_total < wide // 4:
                # the frontier was narrow a round ago: the exact sizes of this
                # one (an all-gather the switch needs anyway) decide
                sizes_n = [x[0] for x in ex.gather_small([nn])]
                total = sum(sizes_n)
                if total < wide // 4:
                    # narrow again: every rank takes the whole frontier
                    configs += total
                    nn_local = 0
                    phase_rounds = 0
                    mine = torch.empty(max(1, nn * cb), dtype=torch.uint8, device=device)
                    if nn:
                        ds.frontier_pack(mine)
                    full = ex.gather_frontier(mine, [x * cb for x in sizes_n])
                    ds.frontier_load(full, total)
                    keep = [full]
                    replicated = True
                    if total == 0:
                        verdict = Illegal
                        break
        wall = time.perf_counter() - t0
        info = ds.info()
        stats = ex.gather_small([int(found and verdict == Ok), info.found_parent, info.found_move, info.found_p4,
                                 info.children, info.max_frontier, int(info.device_ms * 1e3)])
        res = DistResult(verdict=verdict, rounds=rounds, configs=configs, children=sum(s[4] for s in stats),
                         max_frontier=max(s[5] for s in stats), device_ms=max(s[6] for s in stats) / 1e3,
                         wall_s=wall, exchanged_bytes=sent_bytes, per_rank_configs=[part_rounds],
                         xreruns=xreruns, part_s=part_s)
        if verdict == Ok and witness:
            src = next(s for s in stats if s[0])
            traces = ex.gather_traces(ds.trace())
            moves = _walk(traces, src[1], src[2])
            ok = False
            ids = None
            if moves is not None and len(moves) == rounds:
                n_ops = history.info()["n_ops"]
                mv = (ctypes.c_uint32 * max(1, len(moves)))(*moves)
                out = (ctypes.c_int64 * max(1, n_ops))()
                ok = lib().s2lc_witness_from_moves(history._h, mv, len(moves), src[3], out, n_ops) == 0
                ids = list(out[:n_ops]) if ok else None
            res.witness, res.witness_valid = ids, ok
        return res
    finally:
        ds.close()
        del keep
