"""Per-level busy time of each kernel family in a factorisation replay trace
(diagnostics; complements scripts/level_summary.py, same segmentation at the
levels' tile-assembly launches).

    python scripts/level_families.py OUT/.../t_kernel_trace.csv[.gz]
"""
import csv
import gzip
import sys
from collections import defaultdict

path = sys.argv[1]
rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
ev = []
for r in rows:
    name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
    fam = name.split("(")[0].split("<")[0].replace("void ", "").replace("pgo::", "").strip()
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam))
ev.sort()
starts = [i for i, x in enumerate(ev) if x[2] == "k_perm_in"]
ev = ev[starts[-1] if starts else 0:]
end = max(e for _, e, _ in ev)
cuts = [i for i, x in enumerate(ev) if x[2] == "k_assemble_tile"] + [len(ev)]
for li in range(len(cuts) - 1):
    seg = ev[cuts[li]:cuts[li + 1]]
    t0 = seg[0][0]
    t1 = ev[cuts[li + 1]][0] if cuts[li + 1] < len(ev) else end
    busy = defaultdict(float)
    for s, e, f in seg:
        busy[f] += (e - s) / 1e3
    fams = " ".join(f"{k.replace('k_', '')}:{v:.0f}" for k, v in sorted(busy.items(), key=lambda x: -x[1]))
    print(f"level {li:2d} span {(t1 - t0) / 1e3:7.1f} us | {fams}")
