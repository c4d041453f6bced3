"""Per-level panel-step breakdown of one factorisation from a rocprofv3 kernel
trace (scripts/gpu_gtrace.sh):  python scripts/steps.py trace.csv.gz [factorisation#]"""
import collections
import csv
import gzip
import sys

rows = list(csv.DictReader(gzip.open(sys.argv[1], "rt")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_perm_in")]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
w = rows[idx[k]:idx[k + 1]]
t0 = int(w[0]["Start_Timestamp"])
S = lambda r: (int(r["Start_Timestamp"]) - t0) / 1e3
E = lambda r: (int(r["End_Timestamp"]) - t0) / 1e3
name = lambda r: r["Kernel_Name"].split("(")[0].replace("pgo::", "")
print(f"factorisation {k} of {len(idx)}: window {E(w[-1]):.0f} us")
# levels start at k_vec_assemble; within a level, time from the level start to the next
lv = [i for i, r in enumerate(w) if name(r).startswith("k_vec_assemble")] + [len(w)]
bw = next((i for i, r in enumerate(w) if name(r).startswith("k_bwd")), len(w))
print(f"before first level {S(w[lv[0]]):.0f} us; solve from {S(w[bw]):.0f} us")
for a, b in zip(lv, lv[1:]):
    b = min(b, bw)
    seg = w[a:b]
    if not seg:
        continue
    d = collections.Counter()
    n = collections.Counter()
    for r in seg:
        d[name(r)] += E(r) - S(r)
        n[name(r)] += 1
    span = (S(w[b]) if b < len(w) else E(seg[-1])) - S(seg[0])
    top = " ".join(f"{kk[2:14]}:{n[kk]}/{v:.0f}" for kk, v in d.most_common(6))
    print(f"level at {S(seg[0]):8.0f} span {span:7.0f} us  steps {n['k_panel_trsm']:3d}  {top}")
