"""Summarise a rocprofv3 kernel trace of factorisation replays
(scripts/replay_trace.py): takes the last replay (from the last k_perm_in),
prints per kernel family the launches, summed busy time, and the time in which
at least one launch of the family was running; plus the replay's span and the
time the GPU ran nothing.

    python scripts/timeline_summary.py OUT/.../t_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    fam = name.split("(")[0].split("<")[0].replace("void ", "").replace("pgo::", "").strip()
    ev.append((s, e, fam))
ev.sort()
starts = [i for i, x in enumerate(ev) if x[2] == "k_perm_in"]
first = starts[-1] if starts else 0
ev = ev[first:]
t0 = ev[0][0]
t1 = max(e for _, e, _ in ev)
fam_busy = defaultdict(float)
fam_n = defaultdict(int)
fam_int = defaultdict(list)
for s, e, f in ev:
    fam_busy[f] += e - s
    fam_n[f] += 1
    fam_int[f].append((s, e))


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


span = t1 - t0
allu = union([(s, e) for s, e, _ in ev])
print(f"replay span {span / 1e6:.3f} ms, GPU idle {(span - allu) / 1e6:.3f} ms, launches {len(ev)}")
for f in sorted(fam_busy, key=lambda k: -fam_busy[k]):
    print(f"{f:22s} n {fam_n[f]:5d}  busy {fam_busy[f] / 1e6:8.3f} ms  covered {union(fam_int[f]) / 1e6:8.3f} ms")
