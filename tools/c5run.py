import sys, time, json
sys.path[:0] = ['.', 'oracle', 'tests']
import s2_verification_amd as s2
from s2_verification_amd import workloads as W
ck = s2.Checker(device=0)
for name in sys.argv[1:]:
    h = W.config_history(name)
    b = ck.batch([h])
    t = time.time(); r = b.check()[0]; el = time.time() - t
    st = b.stats()
    print(json.dumps({"name": name, "verdict": r.verdict, "reason": r.reason, "wall_s": round(el, 3), "witness": r.witness is not None,
                      **{k: st[k] for k in ("kernel_ms", "level_ms", "level_rounds", "level_configs", "level_children", "level_max_frontier")}}), flush=True)
