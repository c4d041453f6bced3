"""Per-level view of the assembly launches in a PGO_PROFILE_DUMP launch timeline."""
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
    if fac == which and f in ("k_assemble_tile", "k_vec_assemble"):
        rows.append((f, int(lv), int(grid), float(st), float(dur), float(by)))
total = 0.0
for f, lv, grid, st, dur, by in rows:
    gbs = by / (dur * 1e-3) / 1e9 if dur > 0 and by > 0 else 0.0
    print("%-16s lv %2d grid %6d start %7.3f dur %.4f ms %7.1f MB %6.0f GB/s" % (f, lv, grid, st, dur, by / 1e6, gbs))
    if f == "k_assemble_tile":
        total += dur
print("k_assemble_tile total %.3f ms" % total)
