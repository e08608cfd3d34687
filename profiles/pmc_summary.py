"""Summarise rocprofv3 PMC passes for one kernel into profiles/pmc_c4.json.

Usage: python profiles/pmc_summary.py <fetch_dir> <write_dir> <out.json> [kernel] [bench.json]
(kernel: a substring of the kernel name, default "pack_kernel<16>"; bench.json:
the profiled bench.py run's line, for the launch's history count)

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, following
MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts 64 B per 128-B request for
wide coalesced reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.
Both are averaged over the dispatches of that kernel in the run.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_digest import src_digest  # noqa: E402


def canonical(name):
    """pack_kernel<16, true> (the 32-byte-record instance, search.h SRec) and
    pack_kernel<16, false> are both the bench's pack_kernel<16>."""
    return re.sub(r", (true|false)>", ">", name)


def per_dispatch(d, counter, kernel, seen):
    vals = defaultdict(float)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if kernel not in canonical(name):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                seen.add(name)
                vals[row.get("Dispatch_Id")] += float(row.get("Counter_Value", 0))
    return list(vals.values())


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "pack_kernel<16>"
    hist = None
    if len(sys.argv) > 5:
        with open(sys.argv[5]) as fh:
            line = [x for x in fh if x.startswith("{")][-1]
        hist = json.loads(line)["roofline"]["histories_per_launch"]
    seen = set()
    fetch = per_dispatch(fetch_dir, "FETCH_SIZE", kernel, seen)
    write = per_dispatch(write_dir, "WRITE_SIZE", kernel, seen)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} counters found (fetch={len(fetch)}, write={len(write)})")
    f = sum(fetch) / len(fetch)
    w = sum(write) / len(write)
    res = {
        "kernel": kernel,
        "instances": sorted(seen),
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
        "hbm_bytes_per_launch": int((2 * f + w) * 1024),
        "src_digest": src_digest("c4"),
        "histories_per_launch": hist,
        "correction": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts 64 B per 128-B read request)",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
