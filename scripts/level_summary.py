"""Per-level split of one factorisation replay (diagnostics): segments a
rocprofv3 kernel trace of scripts/replay_trace.py at the levels' tile-assembly
launches (one per level, on the library stream) and prints, per level, its
span, the launches of each family in it and the k_step cadence (span / steps).

    python scripts/level_summary.py OUT/.../t_kernel_trace.csv
"""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
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
print(f"replay span {(end - ev[0][0]) / 1e6:.3f} ms")
for li in range(len(cuts) - 1):
    seg = ev[cuts[li]:cuts[li + 1]]
    t0 = seg[0][0]
    t1 = ev[cuts[li + 1]][0] if cuts[li + 1] < len(ev) else end
    n = Counter(f for _, _, f in seg)
    steps = n.get("k_step", 0)
    busy = sum(e - s for s, e, f in seg if f == "k_step")
    cad = f" step cadence {(t1 - t0) / 1e3 / steps:6.1f} us (busy {busy / 1e3 / steps:5.1f})" if steps else ""
    fams = " ".join(f"{k}:{v}" for k, v in sorted(n.items()))
    print(f"level {li:2d} span {(t1 - t0) / 1e3:8.1f} us{cad}  {fams}")

# the top level's panel steps: k_step duration, the gap to the previous
# launch that ended before it (launch latency or a join), and the plain-tile
# launches (k_panel_syrk*) that were still running when it started
seg = ev[cuts[-2]:]
steps = [x for x in seg if x[2] == "k_step"]
gaps, durs = [], []
for i, (s, e, _) in enumerate(steps):
    prev_end = max((e2 for s2, e2, f2 in seg if e2 <= s), default=s)
    plain_busy = sum(1 for s2, e2, f2 in seg if f2.startswith("k_panel_syrk") and s2 < s < e2)
    gaps.append((s - prev_end) / 1e3)
    durs.append((e - s) / 1e3)
    if i < 12 or i == len(steps) - 1:
        print(f"  top step {i:3d}: k_step {durs[-1]:6.1f} us, gap {gaps[-1]:5.1f} us, plain running {plain_busy}")
if steps:
    print(f"top level: {len(steps)} steps, k_step mean {sum(durs) / len(durs):.1f} us, gap mean {sum(gaps) / len(gaps):.1f} us, "
          f"cadence {(steps[-1][1] - steps[0][0]) / 1e3 / len(steps):.1f} us")
