"""Split one optimize's GPU time by kernel family (diagnostics): reads a
rocprofv3 kernel trace of `bench.py --steps 1 --warmup 0` with the side lines
off (graph replays included) and takes the kernels from the first
linearisation to the ninth (the timed optimize: 8 linearisations on C3);
prints the span, the kernels' union and busy time per family.

    python scripts/step_split.py OUT/.../t_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    fam = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("pgo::", "").strip()
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam))
ev.sort()
lin = [s for s, e, f in ev if f == "k_linearize_own"]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # which optimize (8 linearisations each)
t0, tend = lin[8 * k], (lin[8 * k + 8] if len(lin) > 8 * k + 8 else ev[-1][1] + 1)
seg = [x for x in ev if t0 <= x[0] < tend]
t1 = max(e for _, e, _ in seg)
busy = defaultdict(float)
n = defaultdict(int)
for s, e, f in seg:
    busy[f] += e - s
    n[f] += 1


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if cs is not None else 0)


print(f"span {(t1 - t0) / 1e6:.2f} ms, kernels busy (union) {union([(s, e) for s, e, _ in seg]) / 1e6:.2f} ms")
for f in sorted(busy, key=lambda k: -busy[k]):
    print(f"{f:24s} n {n[f]:6d} busy {busy[f] / 1e6:8.2f} ms")
