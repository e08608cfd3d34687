"""Time the level search on named single histories (workloads.CONFIGS), cold
(first run: level buffers allocated) and warm; one JSON line per history.
    python tools/c5run.py C5 C5bad H212"""
import ctypes
import json
import os
import sys
import time

sys.path[:0] = ['.', 'oracle', 'tests']
import s2_verification_amd as s2  # noqa: E402

# S2LC_EXIT_HOOK=1 (profiling the cooperative launches under rocprofv3): end
# the process after the profiler's finalization without the HIP runtime's
# faulting destructor (tools/exit_hook.c). Registered after the
# HIP runtime library is loaded (its destructor then runs after the hook, i.e.
# never) and before the first HIP call (the profiler's finalization handler,
# registered at that call, runs before the hook).
_hook = None
if os.environ.get("S2LC_EXIT_HOOK") == "1":
    s2.lib()
    _hook = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "exit_hook.so"))
    _hook.exit_hook_register()
    _hook.exit_hook_code(1)  # (until the run completes)
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
                                            "level_max_frontier", "level_narrow_ms", "level_wide_ms", "level_solo_ms",
                                            "level_solo_rounds")}}), flush=True)

# release the batches and the context while the HIP runtime is fully up
del b, ck
import gc  # noqa: E402
gc.collect()
if _hook is not None:
    _hook.exit_hook_code(0)
