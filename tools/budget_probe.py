"""Probe: the configuration budget tripping inside a stretch of
one-configuration rounds (H174), per level-search mode (diagnostics)."""
import json
import os
import subprocess
import sys

sys.path[:0] = ['.', 'oracle', 'tests']
MODES = {"default": {}, "no_solo": {"S2LC_NO_SOLO": "1"}, "no_persist": {"S2LC_NO_PERSIST": "1"}}

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import s2_verification_amd as s2
    from s2_verification_amd import workloads as W
    want = json.load(open("tests/golden/hard_round_counts.json"))["H174"]["0"]["counts"]
    r = next(i for i in range(5000, len(want) - 20) if all(c == 1 for c in want[i - 20:i + 20]))
    cum = sum(want[:r + 1])
    h = W.config_history("H174")
    for mc in (cum - 1, cum, cum + 1):
        c = s2.Checker(round_counts=True, max_configs=mc, engine=s2.ENGINE_LEVEL)
        b = c.batch([h])
        res = b.check(with_witness=False)[0]
        got = b.round_counts(0)
        print(json.dumps({"mode": sys.argv[2], "r": r, "cum": cum, "max_configs": mc, "verdict": str(res.verdict),
                          "reason": res.reason, "rounds": res.rounds, "n_counts": len(got),
                          "prefix_ok": got == want[:len(got)], "tail": got[-3:]}), flush=True)
    sys.exit(0)

for m, env in MODES.items():
    subprocess.run([sys.executable, __file__, "--child", m], env={**os.environ, **env}, check=True, timeout=120)
