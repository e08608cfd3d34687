"""Component model of the distributed single-history search on N GPUs
("N-GPU model"), from one-GPU measurements.

    python tools/dist_model.py [--name C5wide] [--ell 10,30,60]

T_N(W) = T_1 - sum_{r in P(W)} t1(r) + sum_{r in P(W)} tau_N(r) + n_sw(W) * sigma

  P(W)    rounds the search partitions with threshold W: from a frontier of
          W configurations on, back to replicated below W / 4 (the rule of
          distributed.check_distributed), on the committed per-round counts
          (tests/golden/hard_round_counts.json)
  t1(r)   the single-GPU engine's time of round r: measured per round from a
          kernel trace of its host-enqueued rounds (profiles/r05/dist/
          <name>_single_kernel_trace.csv: lv_round + lv_insert, matched to
          rounds by replaying the engine's batching policy); rounds inside the
          persistent kernel at its average narrow grid round
  tau_N   max(h, o1 + ell_N + t1(r) / N + x_N(r)): h the host loop per
          partitioned round, o1 the one-GPU overhead of a partitioned round
          over the same round in the single engine (measured, every round
          partitioned: profiles/r05/dist/overhead_wide0.txt), ell_N the RCCL
          all-to-all latency over xGMI (NOT measurable on one GPU: a
          parameter), x_N the transfer of this rank's blocks to the N - 1
          others (the round's new configurations x 2 capacity padding, 640 B
          each at NQ = 4, over 7 links x 50 GB/s)
  sigma   one replicated -> partitioned -> replicated cycle (keep, gather,
          reload into the persistent kernel), from the one-GPU rehearsal:
          (T_rehearsal - T_1 - |P| o1) / cycles
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R5 = os.path.join(ROOT, "profiles", "r05", "dist")


def host_rounds(counts, persist_nf=1024):
    """Rounds the single-GPU engine enqueues from the host (level.hip run
    loop): after a persistent launch ends on a frontier above persist_nf,
    batches of 16 rounds (1 above 4,096) until a batch ends at or below it."""
    out, r, n = [], 1, len(counts)
    nf_last = counts[0]
    while r < n:
        if nf_last <= persist_nf:
            while r < n and counts[r - 1] <= persist_nf:
                r += 1  # (persistent rounds)
            if r >= n:
                break
            r += 1      # the round that outgrew the launch ran inside it
            nf_last = counts[r - 2] if r - 2 < n else 0
            continue
        batch = 16 if nf_last < 4096 else 1
        for _ in range(batch):
            if r >= n:
                break
            out.append(r)
            r += 1
        nf_last = counts[r - 2]
    return out


def partitioned(counts, W, depth=2):
    """Rounds partitioned with threshold W, as distributed._partitioned_rounds
    runs them: from the round after the frontier reaches W; the host reads a
    round's status `depth` rounds late, so the phase ends `depth` rounds after
    the first round (past the phase's second) that expanded a global frontier
    below W / 4."""
    P, r, n = [], 1, len(counts)
    while r < n:
        if counts[r - 1] < W:
            r += 1
            continue
        # counts[r - 1] >= W: round r is the phase's first
        r0 = r
        while r < n:
            P.append(r)
            if r > r0 + 1 and counts[r - 1] < W // 4:
                for k in range(1, depth + 1):
                    if r + k < n:
                        P.append(r + k)
                r += depth + 1
                break
            r += 1
    return P


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="C5wide")
    ap.add_argument("--ell", default="10,30,60", help="RCCL all-to-all latencies to model (us)")
    ap.add_argument("--o1", type=float, default=22.0, help="one-GPU partitioned-round overhead (us)")
    ap.add_argument("--host", type=float, default=27.0, help="host loop per partitioned round (us, upper bound)")
    a = ap.parse_args()
    counts = json.load(open(os.path.join(ROOT, "tests", "golden", "hard_round_counts.json")))[a.name]["0"]["counts"]
    run = json.loads(open(os.path.join(R5, f"{a.name.lower()}_single_run.jsonl")).readline())
    T1 = run["warm_s"] * 1e3
    # per-round times of the host-enqueued rounds (second search of the trace)
    rows = list(csv.DictReader(open(os.path.join(R5, f"{a.name.lower()}_single_kernel_trace.csv"))))
    ev = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"]) for x in rows)
    ks = [("r" if "lv_round" in n else "i" if "lv_insert" in n else "p", s, e) for s, e, n in ev
          if "lv_round" in n or "lv_insert" in n or "lv_persist" in n]
    cut = max(range(len(ks) - 1), key=lambda i: ks[i + 1][1] - ks[i][2]) + 1
    ks = ks[cut:]
    per = [(ks[k][2] - ks[k][1] + (ks[k + 1][2] - ks[k + 1][1] if k + 1 < len(ks) and ks[k + 1][0] == "i" else 0)) / 1e3
           for k in range(len(ks)) if ks[k][0] == "r"]
    per = per[1:]  # (round 0: the initial closure)
    hr = host_rounds(counts)
    assert len(hr) == len(per), (len(hr), len(per))
    t1 = dict(zip(hr, per))
    persist_ms = sum(e - s for n, s, e in ks if n == "p") / 1e6
    solo_ms, solo_rounds = run["level_solo_ms"], run["level_solo_rounds"]
    grid_narrow = max(1, len(counts) - 1 - len(hr) - solo_rounds)
    t_narrow = 1e3 * max(0.0, persist_ms - solo_ms) / grid_narrow  # us per persistent grid round
    rehearsal = {}
    for line in open(os.path.join(R5, "selfx_widths.jsonl")):
        d = json.loads(line)
        if d["name"] == a.name and d["rep"] > 0:
            rehearsal.setdefault(d["wide"], []).append(d["wall_s"] * 1e3)
    print(f"{a.name}: T_1 = {T1:.2f} ms; {len(hr)} host-enqueued rounds (per-round times from the trace), "
          f"persistent grid rounds ~{t_narrow:.1f} us, {solo_rounds} solo rounds")
    ells = [float(x) for x in a.ell.split(",")]
    for W in sorted(set([1024, 4096, 8192, 16384, 32768] + list(rehearsal))):
        P = partitioned(counts, W)
        cycles = sum(1 for i, r in enumerate(P) if i == 0 or P[i - 1] != r - 1)
        t1P = sum(t1.get(r, t_narrow) for r in P) / 1e3
        sig = None
        if W in rehearsal:
            reh = min(rehearsal[W])
            sig = max(0.0, (reh - T1 - len(P) * a.o1 / 1e3) / max(1, cycles))
        s = sig if sig is not None else 0.05
        line = [f"W={W:6d}: |P|={len(P):3d} cycles={cycles:2d} t1(P)={t1P:6.2f} ms"]
        if W in rehearsal:
            line.append(f"rehearsal(1 GPU)={min(rehearsal[W]):.2f} ms sigma={sig * 1e3:.0f} us")
        for N in (2, 4, 8):
            for ell in ells:
                tau = 0.0
                for r in P:
                    x = counts[r] * 640 * 2 * (N - 1) / N / N / 350e3  # us (B/us = 350e3 at 350 GB/s)
                    tau += max(a.host, a.o1 + ell + t1.get(r, t_narrow) / N + x)
                TN = T1 - t1P + tau / 1e3 + cycles * s
                line.append(f"N={N} ell={ell:.0f}: {TN:.2f} ms ({T1 / TN:.3f}x)")
        print("  " + " | ".join(line))


if __name__ == "__main__":
    main()
