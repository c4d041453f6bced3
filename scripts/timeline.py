"""Per-level / per-step view of a PGO_PROFILE_DUMP launch timeline (one factorisation)."""
import collections
import sys

path, which = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows, fac = [], -1
for line in open(path):
    if line.startswith("# factorisation"):
        fac += 1
        continue
    if line.startswith("#"):
        if fac == which:
            print(line.strip())
        continue
    f, lv, kb, grid, st, dur, fl, by = line.split()
    if fac == which:
        rows.append((f, int(lv), int(kb), int(grid), float(st), float(dur), float(fl)))
fac_rows = [r for r in rows if not r[0].startswith("k_bwd") and not (r[0].startswith("k_perm") and r[4] > 1)]
print("factor end %.3f ms, solve end %.3f ms" % (max(r[4] + r[5] for r in fac_rows), max(r[4] + r[5] for r in rows)))
by = collections.defaultdict(list)
for r in fac_rows:
    by[r[1]].append(r)
for lv in sorted(by):
    L = by[lv]
    s, e = min(r[4] for r in L), max(r[4] + r[5] for r in L)
    fam = collections.Counter()
    for r in L:
        fam[r[0]] += r[5]
    print("lv %2d start %7.3f dur %6.3f steps %3d  " % (lv, s, e - s, len(set(r[2] for r in L if r[2] > 0))) +
          " ".join("%s:%.2f" % (k.replace("k_", ""), v) for k, v in fam.most_common(5)))
for lv in [int(x) for x in sys.argv[3:]]:
    print("level", lv)
    for r in sorted(by[lv], key=lambda r: r[4])[:24]:
        print("   %-18s kb %3d grid %5d start %7.3f dur %6.3f" % (r[0], r[2], r[3], r[4], r[5]))
