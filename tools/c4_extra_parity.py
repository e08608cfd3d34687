"""C4-shaped histories beyond the committed 10k batch (DST seeds a .. b-1,
workloads.c4_params: 5-8 clients x 100 ops, three workflows, every 10th seed
with an injected violation): GPU verdicts + certified witnesses against the
CPU oracle (porcupine's WGL restated, oracle/oracle.c) checked in parallel
processes. One JSON line: counts and any mismatching seeds.

    python tools/c4_extra_parity.py [first_seed] [n] [procs] [clients]   (default 10000 50000 16 -)
clients: num_clients = clients + seed % 8 instead of C4's 5 + seed % 4 (wider
histories: the 32-lane packed kernel and the workgroup engine).
"""
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def _params(sd, clients):
    from s2_verification_amd import workloads as W
    kw = W.c4_params(sd)
    if clients:
        kw["num_clients"] = clients + sd % 8
    return kw


def _oracle(seeds, clients=0):
    import oracle as orc
    import s2_verification_amd as s2
    out = []
    for sd in seeds:
        h = s2.simulate_history(**_params(sd, clients))
        v, _ = orc.check_wgl(orc.from_s2lc_numpy(h.events_numpy(), owner=h), timeout=60.0)
        out.append((sd, v))
    return out


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    procs = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    clients = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] != "-" else 0
    seeds = list(range(first, first + n))
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        chunks = [(seeds[i:i + 200], clients) for i in range(0, n, 200)]
        async_res = pool.starmap_async(_oracle, chunks, chunksize=1)
        import numpy as np
        import s2_verification_amd as s2
        hs = [s2.simulate_history(**_params(sd, clients)) for sd in seeds]
        b = s2.Checker().batch(hs)
        b.run()
        flat = b.results_flat(with_witness=True)  # raises on any witness that fails CPU replay
        gpu_t = time.perf_counter() - t0
        print(json.dumps({"gpu_phase_s": round(gpu_t, 1)}), file=sys.stderr, flush=True)
        while not async_res.ready():  # a progress line a minute (the oracle side can run for minutes)
            async_res.wait(50)
            print(json.dumps({"oracle_running_s": round(time.perf_counter() - t0, 1)}), file=sys.stderr, flush=True)
        ref = dict(x for part in async_res.get() for x in part)
    names = {s2.S2LC_OK: "Ok", s2.S2LC_ILLEGAL: "Illegal"}
    got = [names.get(int(v), "Unknown") for v in flat["verdict"]]
    wl = np.diff(flat["witness_offs"].astype(np.int64))
    n_ops = np.array([h.info()["n_ops"] for h in hs], np.int64)
    bad = [sd for sd, g in zip(seeds, got) if ref[sd] != "Unknown" and g != ref[sd]]
    unknown_oracle = sum(1 for sd in seeds if ref[sd] == "Unknown")
    okw = [i for i, g in enumerate(got) if g == "Ok" and wl[i] != n_ops[i]]
    st = b.stats()
    print(json.dumps({"first_seed": first, "histories": n, "clients": clients or "c4", "oracle_procs": procs,
                      "pack16": st["pack16_histories"], "pack8": st["pack8_histories"], "level": st["level_histories"],
                      "gpu_ok": got.count("Ok"), "gpu_illegal": got.count("Illegal"),
                      "gpu_unknown": got.count("Unknown"), "oracle_unknown": unknown_oracle,
                      "verdict_mismatches": len(bad), "mismatch_seeds": bad[:20],
                      "ok_without_full_certified_witness": len(okw),
                      "seconds": round(time.perf_counter() - t0, 1), "gpu_phase_s": round(gpu_t, 1)}), flush=True)
    return 0 if not bad and not okw else 1


if __name__ == "__main__":
    sys.exit(main())
