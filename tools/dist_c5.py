"""Time the distributed single-history search (one process per rank).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        tools/dist_c5.py [--backend nccl|gloo] [--wide W] [names...]
With gloo every rank may share GPU 0 (protocol rehearsal on a 1-GPU box).
"""
import argparse
import json
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402
from s2_verification_amd.distributed import bind_stream, check_distributed  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--backend", default="nccl")
ap.add_argument("--wide", type=int, default=4096)
ap.add_argument("--selfx", action="store_true", help="one rank: partitioned rounds through a self-exchange")
ap.add_argument("--sized", action="store_true", help="partitioned rounds the round-3 way (host-read sizes)")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--xcap0", type=int, default=0, help="first exchange block capacity (0: from the frontier)")
ap.add_argument("names", nargs="*", default=["C5"])
a = ap.parse_args()
rank = int(os.environ.get("RANK", 0))
local = int(os.environ.get("LOCAL_RANK", 0))
dev = local if a.backend == "nccl" else 0
torch.cuda.set_device(dev)
if a.backend == "nccl":
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
else:
    dist.init_process_group("gloo")
ck = s2.Checker(device=dev, stream=bind_stream() if a.backend == "nccl" else 0)
for name in a.names:
    h = W.config_history(name)
    for rep in range(a.reps):
        r = check_distributed(ck, h, wide=a.wide, self_exchange=a.selfx, sized_exchange=a.sized,
                              xcap0=a.xcap0 or None)
        if rank != 0:
            continue
        pr = r.per_rank_configs[0]
        print(json.dumps({"name": name, "rep": rep, "world": dist.get_world_size(), "backend": a.backend,
                          "wide": a.wide, "selfx": a.selfx, "sized": a.sized,
                          "verdict": r.verdict, "witness_valid": r.witness_valid, "wall_s": round(r.wall_s, 4),
                          "rounds": r.rounds, "partitioned_rounds": pr, "part_s": round(r.part_s, 4),
                          "us_per_partitioned_round": round(1e6 * r.part_s / pr, 1) if pr else None,
                          "xreruns": r.xreruns, "configs": r.configs,
                          "children": r.children, "device_ms_max": round(r.device_ms, 1),
                          "sent_bytes_rank0": r.exchanged_bytes}), flush=True)
dist.destroy_process_group()
