"""Summarise the rocprofv3 PMC passes of profiles/collect_pmc.sh.

Usage: python profiles/pmc_sq.py gpurun_out/<tag>
Per pass directory and kernel: counter sums per dispatch, averaged over the
kernel's dispatches, plus derived figures:
  issue_frac   = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (waves issuing)
  wait_frac    = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  stall_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls)
  avg_waves    = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES (resident waves per busy SQ cycle, chip-wide sum / 8 XCDs)
  hbm_bytes    = (2 * FETCH_SIZE + WRITE_SIZE) KiB (MI355X_MICROARCH.md gfx950 correction)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KERNELS = ["pack_kernel<8>", "pack_kernel<16>", "lv_persist", "lv_round", "lv_insert", "walk_kernel", "search_kernel"]


def kname(n):
    for k in KERNELS:
        base = k.split("<")[0]
        if base not in n:
            continue
        if k == base:
            return k
        arg = k[len(base) + 1:-1]
        if f"<{arg}>" in n or f"<{arg}," in n or f"ILi{arg}E" in n:
            return k
    m = re.search(r"(\w+_kernel|lv_\w+)", n)
    return m.group(1) if m else n[:40]


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                key = (kname(row.get("Kernel_Name", "")), row.get("Dispatch_Id"))
                per[key][row["Counter_Name"]] += float(row.get("Counter_Value", 0) or 0)
    out = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            out[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": max(len(v) for v in cs.values())}
            | {c + "_total": sum(v) for c, v in cs.items() if c.startswith("TCC_")}
            for k, cs in out.items()}


def derive(c):
    d = {}
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for num, name in (("SQ_ACTIVE_INST_ANY", "issue_frac"), ("SQ_WAIT_ANY", "wait_frac"),
                          ("SQ_WAIT_INST_ANY", "stall_frac")):
            if num in c:
                d[name] = round(c[num] / wc, 4)
        if c.get("SQ_BUSY_CYCLES"):
            d["avg_waves"] = round(wc / c["SQ_BUSY_CYCLES"], 2)
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        d["hbm_bytes_part"] = int((2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024)
    return d


def main():
    root = sys.argv[1]
    res = {}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(d):
            continue
        stats = load(d)
        if not stats:
            continue
        res[os.path.basename(d)] = {k: {**{c: round(v, 1) for c, v in cs.items()}, **derive(cs)}
                                    for k, cs in stats.items() if k in KERNELS}
        tot = {}
        for k, cs in stats.items():
            for c, v in cs.items():
                if c.endswith("_total") and k.startswith("lv_"):
                    tot[c] = tot.get(c, 0.0) + v
        if tot:
            res[os.path.basename(d)]["level_search_totals"] = {c: round(v, 1) for c, v in tot.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
