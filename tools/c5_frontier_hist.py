import sys, json, collections
sys.path[:0] = ['.']
import numpy as np
import s2_verification_amd as s2
from s2_verification_amd import workloads as W
for name in sys.argv[1:]:
    h = W.config_history(name)
    c = s2.Checker(round_counts=True)
    b = c.batch([h])
    r = b.check()[0]
    rc = np.array(b.round_counts(0), dtype=np.int64)
    edges = [0, 1, 2, 5, 17, 65, 257, 1025, 4097, 16385, 65537, 1 << 40]
    hist = np.histogram(rc, bins=edges)[0]
    print(json.dumps({"name": name, "rounds": int(len(rc)), "hist": {f"{edges[i]}-{edges[i+1]-1}": int(hist[i]) for i in range(len(hist))},
                      "configs_in_2_4096": int(rc[(rc >= 2) & (rc <= 4096)].sum())}))
