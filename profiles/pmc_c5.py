"""C5 roofline counters from the rocprofv3 PMC passes (profiles/collect_pmc.sh:
c5_fetch, c5_write, c5_atomic over tools/c5run.py C5 = two searches, cold +
warm), per search, summed over the level-search kernels (lv_*):
  hbm_bytes_per_search       = (2 * FETCH_SIZE + WRITE_SIZE) KiB (gfx950 correction,
                               MI355X_MICROARCH.md)
  tcc_ea_atomics_per_search  = TCC_EA0_ATOMIC (device-scope atomics reaching memory)
Usage: python profiles/pmc_c5.py gpurun_out/<tag> > profiles/<round>/pmc_c5.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_sq import load  # noqa: E402
from kernel_digest import src_digest  # noqa: E402

SEARCHES = 2


def lv_total(stats, counter):
    return sum(cs.get(counter + "_total", cs.get(counter, 0.0) * cs.get("dispatches", 1))
               for k, cs in stats.items() if k.startswith("lv_"))


def per_kernel(fetch, write, atom):
    """Each lv_ kernel's counters from all three passes, per search (MiB for
    the sizes; the gfx950 FETCH_SIZE correction applied)."""
    out = {}
    for k in sorted(set(fetch) | set(write) | set(atom)):
        if not k.startswith("lv_"):
            continue
        f, w, a = fetch.get(k, {}), write.get(k, {}), atom.get(k, {})
        out[k] = {"dispatches": f.get("dispatches", w.get("dispatches", a.get("dispatches", 0))),
                  "fetch_MiB_per_search": round(2 * f.get("FETCH_SIZE", 0.0) * f.get("dispatches", 0) / 1024 / SEARCHES, 1),
                  "write_MiB_per_search": round(w.get("WRITE_SIZE", 0.0) * w.get("dispatches", 0) / 1024 / SEARCHES, 1),
                  "atomics_per_search": round(a.get("TCC_EA0_ATOMIC_total", 0.0) / SEARCHES, 1)}
    return out


def main():
    root = sys.argv[1]
    fetch = load(os.path.join(root, "c5_fetch"))
    write = load(os.path.join(root, "c5_write"))
    atom = load(os.path.join(root, "c5_atomic"))
    # FETCH_SIZE / WRITE_SIZE are derived (not TCC_ prefixed): per-dispatch averages x dispatches
    fb = sum(cs.get("FETCH_SIZE", 0.0) * cs["dispatches"] for k, cs in fetch.items() if k.startswith("lv_"))
    wb = sum(cs.get("WRITE_SIZE", 0.0) * cs["dispatches"] for k, cs in write.items() if k.startswith("lv_"))
    out = {
        "workload": "C5 (tools/c5run.py C5: two searches, cold + warm)",
        "kernels": "lv_persist + lv_round + lv_insert",
        "src_digest": src_digest("c5"),
        "hbm_bytes_per_search": round((2 * fb + wb) * 1024 / SEARCHES, 1),
        "tcc_ea_atomics_per_search": round(lv_total(atom, "TCC_EA0_ATOMIC") / SEARCHES, 1),
        "tcc_atomics_per_search": round(lv_total(atom, "TCC_ATOMIC") / SEARCHES, 1),
        "per_kernel": per_kernel(fetch, write, atom),
        "source": "rocprofv3 --pmc passes (profiles/collect_pmc.sh: c5_fetch FETCH_SIZE TCC_ATOMIC, "
                  "c5_write WRITE_SIZE TCC_ATOMIC, c5_atomic TCC_ATOMIC TCC_EA0_ATOMIC)",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
