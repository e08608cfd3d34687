"""C4-shaped collector JSONL for tools/decode_prof/prof (length-prefixed blobs)."""
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402

out, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 500
with open(out, "wb") as f:
    for sd in range(2 * 10 ** 6, 2 * 10 ** 6 + n):
        b = s2.simulate_jsonl(**W.c4_params(sd))
        f.write(struct.pack("<Q", len(b)) + b)
