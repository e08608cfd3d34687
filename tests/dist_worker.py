"""Worker processes for the multi-rank tests (spawned; one per rank)."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def _init(rank, world, port, backend):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group(backend, rank=rank, world_size=world)
    return dist


def exchange_worker(rank, world, port, q):
    """CPU (gloo): the round's small all-to-all and the trace gather."""
    try:
        import numpy as np
        import torch
        from s2_verification_amd.distributed import _Exchange, _walk
        dist = _init(rank, world, port, "gloo")
        ex = _Exchange(None, torch.device("cpu"))
        counts = [10 * rank + w for w in range(world)]  # rank -> w
        recv, found_any, staged, front = ex.counts(counts, rank == world - 1, sum(counts), 100 + rank)
        assert front == sum(100 + r for r in range(world))
        tr = np.array([[0xFFFFFFFF, 0xFFFFFFFF], [(rank << 29) | 0, rank + 1]], dtype=np.uint32)
        traces = ex.gather_traces(tr)
        # fixed-capacity blocks to the other ranks (no sizes, no own block):
        # the block for rank w of rank r's send buffer holds bytes (r, w, 0, 1,
        # ...); the block from rank s of what rank r receives is what s sent to r
        blk = 24
        others = [w for w in range(world) if w != rank]
        send = torch.zeros(len(others) * blk, dtype=torch.uint8)
        for b, w in enumerate(others):
            send[b * blk:(b + 1) * blk] = torch.tensor([rank, w] + list(range(blk - 2)), dtype=torch.uint8)
        got = ex.payload_blocks(send, blk)
        blocks = [got[b * blk:(b + 1) * blk].tolist()[:2] for b in range(len(others))]
        q.put((rank, recv, found_any, staged, [t.tolist() for t in traces], blocks))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "error", traceback.format_exc()))


def search_worker(rank, world, port, backend, names, wide, persistent, self_exchange, q, sized=False, xcap0=None,
                  stream_mode=None):
    """GPU: every rank checks the named histories with check_distributed.
    stream_mode: "bound" (the library on torch's current stream: nccl's
    default), "own" (the library's own stream: gloo's default) or "side" (a
    caller stream that is NOT torch's current one: the collectives and the
    library's kernels are ordered by stream waits)."""
    try:
        import torch
        import s2_verification_amd as s2
        from s2_verification_amd import workloads as W
        from s2_verification_amd.distributed import bind_stream, check_distributed
        torch.cuda.set_device(0 if backend == "gloo" else rank)
        dist = _init(rank, world, port, backend)
        # nccl: the library on torch's stream (no host syncs around the collectives)
        mode = stream_mode or ("bound" if backend == "nccl" else "own")
        side = torch.cuda.Stream() if mode == "side" else None
        stream = bind_stream() if mode == "bound" else side.cuda_stream if side is not None else 0
        checker = s2.Checker(device=torch.cuda.current_device(), stream=stream)
        out = []
        for name in names:
            h = W.config_history(name)
            r = check_distributed(checker, h, wide=wide, persistent=persistent, self_exchange=self_exchange,
                                  sized_exchange=sized, xcap0=xcap0)
            out.append((name, r.verdict, r.rounds, r.configs, r.witness_valid,
                        None if r.witness is None else len(r.witness), h.info()["n_ops"], r.xreruns,
                        r.per_rank_configs[0]))
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "error", traceback.format_exc()))


def overflow_worker(rank, world, port, backend, name, wide, scap, q):
    """GPU: an exchanged round whose winners (the rank's own share
    plus the received blocks) can pass the staging capacity, with the witness
    on: a staging array forced small (S2LC_LEVEL_SCAP, read when the level
    buffers are first sized). The search must end cleanly (a verdict, or the
    buffer error), never write past its trace pool; a second history checked
    afterwards in the same process must still be right."""
    try:
        os.environ["S2LC_LEVEL_SCAP"] = str(scap)
        import torch
        import s2_verification_amd as s2
        from s2_verification_amd import workloads as W
        from s2_verification_amd.distributed import check_distributed
        torch.cuda.set_device(0 if backend == "gloo" else rank)
        dist = _init(rank, world, port, backend)
        checker = s2.Checker(device=torch.cuda.current_device())
        out = []
        try:
            r = check_distributed(checker, W.config_history(name), wide=wide, persistent=False, witness=True)
            out.append(("verdict", r.verdict, r.rounds, r.witness_valid))
        except s2.S2LCError as e:
            out.append(("error", str(e)))
        # the process (and its device) is still sound: the single-GPU engine
        # on a small history
        h = W.config_history("C1")
        rr = checker.check(h)
        out.append(("after", rr.verdict, rr.witness is not None))
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "error", traceback.format_exc()))
