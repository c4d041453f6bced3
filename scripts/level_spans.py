"""Per-level spans (us) of one-lane / three-lane replays from
scripts/gpu_levels.sh output (levels_l1.txt, levels_l3.txt) into
profiles/<out>.json, which graphslam_amd/multi_model.py reads.

    python scripts/level_spans.py gpurun_out/levels_TAG [--config C3] [--out r04_level_spans]
"""
import argparse
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--config", default="C3")
ap.add_argument("--out", default="r04_level_spans")
args = ap.parse_args()
res = {}
for lanes in (1, 3):
    spans = []
    for line in open(os.path.join(args.dir, f"levels_l{lanes}.txt")):
        m = re.match(r"level\s+(\d+) span\s+([\d.]+) us", line)
        if m:
            spans.append(float(m.group(2)))
    res[str(lanes)] = spans
out = {args.config: res,
       "source": f"rocprofv3 kernel traces of factorisation graph replays (scripts/gpu_levels.sh, "
                 f"{os.path.basename(args.dir.rstrip('/'))}; scripts/level_summary.py), us per level"}
path = os.path.join(ROOT, "profiles", args.out + ".json")
json.dump(out, open(path, "w"), indent=1)
print("wrote", path, {k: round(sum(v), 1) for k, v in res.items()})
