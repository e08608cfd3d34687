"""Digest of the device-code sources a PMC pass measured, so bench.py reports
`roofline.traffic` only from a PMC summary of the kernels it is running
(a stale committed PMC file must not pass for this run's
traffic).

    c4: the packed/workgroup search kernels (pack_kernel, search_kernel)
    c5: the level search (lv_persist, lv_round, lv_insert)
"""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "s2_verification_amd", "csrc")
FILES = {
    "c4": ("model.h", "search.h", "search_dev.h", "pack_dev.h", "search.hip"),
    "c5": ("model.h", "search.h", "level_dev.h", "solo_dev.h", "level.hip"),
}


def src_digest(kind):
    h = hashlib.sha256()
    for name in FILES[kind]:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    for k in FILES:
        print(k, src_digest(k))
