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
from s2_verification_amd.distributed import check_distributed  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--backend", default="nccl")
ap.add_argument("--wide", type=int, default=4096)
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
ck = s2.Checker(device=dev, stream=torch.cuda.current_stream().cuda_stream if a.backend == "nccl" else 0)
for name in a.names:
    h = W.config_history(name)
    r = check_distributed(ck, h, wide=a.wide)
    if rank == 0:
        print(json.dumps({"name": name, "world": dist.get_world_size(), "backend": a.backend, "wide": a.wide,
                          "verdict": r.verdict, "witness_valid": r.witness_valid, "wall_s": round(r.wall_s, 4),
                          "rounds": r.rounds, "partitioned_rounds": r.per_rank_configs, "configs": r.configs,
                          "children": r.children, "device_ms_max": round(r.device_ms, 1),
                          "sent_bytes_rank0": r.exchanged_bytes}), flush=True)
dist.destroy_process_group()
