"""Per-level view of the backward solve in a PGO_PROFILE_DUMP launch timeline."""
import collections
import sys

path, which = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows, fac = [], -1
for line in open(path):
    if line.startswith("# factorisation"):
        fac += 1
        continue
    if line.startswith("#"):
        continue
    f, lv, kb, grid, st, dur, fl, by = line.split()
    if fac == which and (f.startswith("k_bwd") or f.startswith("k_perm")):
        rows.append((f, int(lv), int(grid), float(st), float(dur), float(fl)))
if not rows:
    sys.exit("no backward launches in factorisation %d" % which)
t0 = min(r[3] for r in rows)
print("solve span %.3f ms, summed %.3f ms" % (max(r[3] + r[4] for r in rows) - t0, sum(r[4] for r in rows)))
by = collections.defaultdict(list)
for r in rows:
    by[r[1]].append(r)
for lv in sorted(by, reverse=True):
    for f, _, grid, st, dur, fl in by[lv]:
        gbs = 4.0 * fl / (dur * 1e-3) / 1e9 if f == "k_bwd_part" and dur > 0 else 0.0
        print("lv %2d %-12s grid %6d start %7.3f dur %7.4f ms  %s" % (lv, f, grid, st - t0, dur,
              ("%.0f GB/s" % gbs) if gbs else ""))
