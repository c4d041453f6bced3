"""Print the headline, the factorisation roofline and the per-family table of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.3f it/s  ms/step %.1f" % (d["value"], d["ms_per_step"]), {k: d["per_step"][k] for k in
      ("linearizations", "lm_tries", "lambda_rounds", "ms_solve", "stop_reason")})
r = d["roofline"]
print({k: v for k, v in r.items() if k not in ("families",)})
for k, v in sorted(r.get("families", {}).items(), key=lambda kv: -kv[1]["ms"]):
    print("  %-26s launches %5d  ms %8.3f  avg %.4f  share %.3f  %s %.3f" % (
        k, v["launches"], v["ms"], v["avg_launch_ms"], v["share"], v["unit"], v["achieved"] or 0))
