"""Time the level search on named single histories (workloads.CONFIGS), cold
(first run: level buffers allocated) and warm; one JSON line per history.
    python tools/c5run.py C5 C5bad H212"""
import json
import os
import sys
import time

sys.path[:0] = ['.', 'oracle', 'tests']
import s2_verification_amd as s2  # noqa: E402
from s2_verification_amd import workloads as W  # noqa: E402

ck = s2.Checker(device=0)
for name in sys.argv[1:]:
    h = W.config_history(name)
    b = ck.batch([h])
    t = time.time()
    r = b.check()[0]
    cold = time.time() - t
    t = time.time()
    b.run()
    warm = time.time() - t
    st = b.stats()
    print(json.dumps({"name": name, "verdict": r.verdict, "reason": r.reason, "cold_s": round(cold, 3),
                      "warm_s": round(warm, 4), "witness": r.witness is not None,
                      **{k: st[k] for k in ("kernel_ms", "level_ms", "level_rounds", "level_configs", "level_children",
                                            "level_max_frontier")}}), flush=True)

# Leave without running the libraries' exit-time destructors: under rocprofv3
# --kernel-trace the HIP module destructor of the level-search code object
# faulted inside the HIP runtime after the profiler had finalized and written
# its output (gpurun_out/r03a/c5stats.err); the results above are complete.
sys.stdout.flush()
del ck
os._exit(0)
