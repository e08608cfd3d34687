"""Multi-rank tests of the distributed single-history search (s2_verification_amd.distributed).

CPU (gloo, world 2): the per-round small all-to-all (counts, found, staged
totals) and the trace gather + cross-rank witness walk.
GPU (one MI355X): world 1 and world 2 with both ranks on the same GPU over
gloo (host-staged payload): verdicts equal the committed reduced-search
verdicts, Ok witnesses certified through the CPU model. The RCCL transport
differs only in where the two all-to-alls run (same calls on CUDA tensors).
"""
import multiprocessing as mp
import random

import pytest

from helpers import config_digest, golden


def _spawn(target, args_per_rank, timeout=600, extra=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=a + (q,) + tuple(extra)) for a in args_per_rank]
    for p in ps:
        p.start()
    out = [q.get(timeout=timeout) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert o[1] != "error", o[2]
    return sorted(out, key=lambda o: o[0])


def test_exchange_gloo_world2():
    import dist_worker
    port = random.randint(20000, 40000)
    out = _spawn(dist_worker.exchange_worker, [(r, 2, port) for r in range(2)], timeout=120)
    for rank, recv, found_any, staged, traces, blocks in out:
        assert recv == [10 * s + rank for s in range(2)]  # what each source sent to me
        assert blocks == [[s, rank] for s in range(2) if s != rank]  # fixed-capacity blocks: one from each other rank
        assert found_any is True
        assert staged == sum(10 * s + w for s in range(2) for w in range(2))
        assert traces == [[[0xFFFFFFFF, 0xFFFFFFFF], [(s << 29), s + 1]] for s in range(2)]


def test_walk_crosses_ranks():
    import numpy as np
    from s2_verification_amd.distributed import _walk
    N = 0xFFFFFFFF
    t0 = np.array([[N, N], [(1 << 29) | 0, 5]], dtype=np.uint32)       # rank 0: root, then (parent r1#0, move 5)
    t1 = np.array([[0, 3]], dtype=np.uint32)                          # rank 1: (parent r0#0, move 3)
    assert _walk([t0, t1], parent=1, move=7) == [3, 5, 7]
    assert _walk([t0, t1], parent=N, move=N) == []
    assert _walk([t0, t1], parent=(2 << 29), move=1) is None


@pytest.mark.gpu
@pytest.mark.parametrize("world,wide,backend,persistent,selfx", [
    (1, 4096, "gloo", True, False), (1, 4096, "gloo", False, False),
    (2, 0, "gloo", None, False), (2, 256, "gloo", None, False),
    (3, 1024, "gloo", None, False),
    (1, 0, "nccl", None, False), (1, 4096, "nccl", True, False),
    (1, 256, "nccl", True, True), (1, 1024, "gloo", True, True),
    (2, 256, "gloo", True, False)])
def test_distributed_search_one_gpu(world, wide, backend, persistent, selfx):
    """wide=0: every round partitioned; otherwise replicated while the
    frontier is narrower than `wide`, partitioned above it (both switches
    happen on H212 / C5bad at 256 and 1024); replicated rounds inside the
    persistent kernel (s2lc_dist_local_run) or host-driven one by one. The
    nccl cases are RCCL with one rank: partitioning every round (a
    self-exchange through the same all-to-all calls the multi-GPU run makes),
    the persistent replicated rounds, and (selfx) the multi-GPU sequence
    replicated-in-the-persistent-kernel -> partitioned -> gathered ->
    replicated again on one rank. World 2 with persistent=True: two processes'
    persistent grids on one GPU (cooperative launches, or a barrier time-out
    that sends the search back to host-driven rounds; the verdict and round
    counts must not change)."""
    import dist_worker
    ref = golden("hard_reduced.json")
    names = [n for n in ("H174", "C5bad", "H212") if n in ref]
    port = random.randint(20000, 40000)
    out = _spawn(dist_worker.search_worker, [(r, world, port, backend, names, wide, persistent, selfx)
                                             for r in range(world)])
    rc = golden("hard_round_counts.json")
    for rank, res in out:
        for name, verdict, rounds, configs, wvalid, wlen, n_ops, _, _ in res:
            assert verdict == ref[name]["verdict"], (rank, name, verdict)
            assert rounds == rc[name]["0"]["rounds"], (rank, name, rounds)
            if verdict == "Ok":
                assert wvalid and wlen == n_ops, (rank, name, wvalid, wlen)
    # every rank agrees
    assert len({tuple(r) for _, res in out for r in res}) == len(names)


@pytest.mark.gpu
@pytest.mark.parametrize("world,wide,backend", [(2, 4096, "gloo"), (1, 4096, "nccl"), (1, 0, "nccl")])
def test_distributed_wide_history(world, wide, backend):
    """C5wide: a hard history whose wide rounds hold 93 % of its unique
    configurations (frontier up to 273 k), the shape the partitioned rounds
    split across GPUs: verdict, round count and certified witness against the
    committed CPU reduced search."""
    import dist_worker
    ref = golden("hard_reduced.json")["C5wide"]
    rc = golden("hard_round_counts.json")["C5wide"]["0"]
    assert config_digest("C5wide") == ref["digest"], "simulator output changed: regenerate the fixture"
    port = random.randint(20000, 40000)
    out = _spawn(dist_worker.search_worker, [(r, world, port, backend, ["C5wide"], wide, None, False)
                                             for r in range(world)])
    for rank, res in out:
        for name, verdict, rounds, configs, wvalid, wlen, n_ops, _, _ in res:
            assert verdict == ref["verdict"] and rounds == rc["rounds"], (rank, verdict, rounds)
            assert configs == sum(rc["counts"]), (rank, configs, sum(rc["counts"]))  # (round 0 included)
            assert wvalid and wlen == n_ops, (rank, wvalid, wlen)


@pytest.mark.gpu
@pytest.mark.parametrize("world,wide,backend,sized,xcap0", [
    (2, 256, "gloo", True, None), (1, 0, "nccl", True, None),
    (2, 256, "gloo", False, 1), (1, 256, "nccl", False, 1), (2, 256, "nccl", False, 1)])
def test_partitioned_exchange_modes(world, wide, backend, sized, xcap0):
    """Partitioned rounds the round-3 way (sized: host-read counts and a
    variable-split all-to-all) and host-free with exchange blocks of capacity
    1 at every switch (with 2 ranks every first partitioned round overflows
    its blocks on all ranks, inserts nothing and is re-run with larger ones;
    one rank sends no block at all, its share stays local): H212 and C5bad
    give the committed verdicts and round counts, and C5wide's unique
    configurations sum to the committed total."""
    import dist_worker
    import torch
    if backend == "nccl" and world > torch.cuda.device_count():
        # (the host-free rounds over RCCL with two ranks, one GPU
        # each, forced re-runs included; runs where the box has the GPUs)
        pytest.skip(f"{world} ranks over RCCL need {world} GPUs")
    ref = golden("hard_reduced.json")
    rc = golden("hard_round_counts.json")
    names = ["H212", "C5bad", "C5wide"]
    port = random.randint(20000, 40000)
    out = _spawn(dist_worker.search_worker, [(r, world, port, backend, names, wide, None, world == 1)
                                             for r in range(world)], extra=(sized, xcap0))
    for rank, res in out:
        for name, verdict, rounds, configs, wvalid, wlen, n_ops, xreruns, part in res:
            assert verdict == ref[name]["verdict"], (rank, name, verdict)
            assert rounds == rc[name]["0"]["rounds"], (rank, name, rounds)
            if name == "C5wide":
                assert configs == sum(rc[name]["0"]["counts"]), (rank, configs)
            if verdict == "Ok":
                assert wvalid and wlen == n_ops, (rank, name, wvalid, wlen)
            assert part > 0, (rank, name)
            if xcap0 == 1 and world > 1:
                assert xreruns >= 1, (rank, name, xreruns)
            if world == 1 and not sized:  # (the own share never travels: no block to outgrow)
                assert xreruns == 0, (rank, name, xreruns)
            if sized:
                assert xreruns == 0
    assert len({tuple(r) for _, res in out for r in res}) == len(names)


@pytest.mark.gpu
@pytest.mark.parametrize("world,wide,backend,selfx", [(1, 256, "nccl", True), (2, 256, "gloo", False)])
def test_distributed_search_on_a_side_stream(world, wide, backend, selfx):
    """Checker(stream=X) with X a caller stream that is not torch's
    current one. The library then skips its host waits, so the collectives
    must wait for its queued kernels (and its next kernels for the
    collectives) on the device: verdicts, round counts and certified
    witnesses as committed."""
    import dist_worker
    ref = golden("hard_reduced.json")
    rc = golden("hard_round_counts.json")
    names = ["H212", "C5bad"]
    port = random.randint(20000, 40000)
    out = _spawn(dist_worker.search_worker, [(r, world, port, backend, names, wide, None, selfx)
                                             for r in range(world)], extra=(False, None, "side"))
    for rank, res in out:
        for name, verdict, rounds, configs, wvalid, wlen, n_ops, xreruns, part in res:
            assert verdict == ref[name]["verdict"] and rounds == rc[name]["0"]["rounds"], (rank, name, verdict, rounds)
            assert part > 0, (rank, name)
            if verdict == "Ok":
                assert wvalid and wlen == n_ops, (rank, name, wvalid, wlen)


@pytest.mark.gpu
def test_exchanged_round_past_staging_capacity_with_witness():
    """in an exchanged round lv_insert takes the rank's whole local
    share plus the received blocks, so a round's winners can number more than
    the staging capacity. Those winners get no frontier index and no trace
    entry (the close stops the run). With a staging array forced to 1,024
    configurations, H212's partitioned rounds (2 ranks, from a frontier of
    256) end either with the committed verdict and round count or with the
    capacity error, identically on both ranks, and the process then checks
    another history correctly."""
    import dist_worker
    ref = golden("hard_reduced.json")["H212"]
    port = random.randint(20000, 40000)
    out = _spawn(dist_worker.overflow_worker, [(r, 2, port, "gloo", "H212", 256, 1024) for r in range(2)])
    outcomes = set()
    for rank, res in out:
        first, after = res
        if first[0] == "verdict":
            assert first[1] == ref["verdict"] and first[2] == ref["reduced"]["rounds"], (rank, first)
            if first[1] == "Ok":
                assert first[3], (rank, first)
            outcomes.add(first[:3])
        else:
            assert "exceeds" in first[1] or "frontier" in first[1], (rank, first)
            outcomes.add(("error",))
        assert after[1:] == ("Ok", True), (rank, after)
    assert len(outcomes) == 1, outcomes
