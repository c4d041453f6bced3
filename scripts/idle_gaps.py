"""GPU idle time inside the timed optimize of a rocprofv3 kernel trace
(scripts/gpu_r05o.sh: one warm-up + one timed C3 optimize, graph replays).

    python scripts/idle_gaps.py gpurun_out/r05o/trace [--linearizations 8]

The timed optimize is taken from the (n+1)-th k_linearize_own launch (n = the
linearisations of one optimize) to the last kernel.  Prints the busy time
(union of kernel intervals over every queue), the idle gaps by size, and the
gaps that follow each kernel family (what the GPU waits on: the host's turn
between lambda rounds, event joins, launches).
"""
import argparse
import collections
import csv
import glob
import gzip
import json
import os


def load(d):
    f = (glob.glob(os.path.join(d, "**", "*kernel_trace.csv.gz"), recursive=True) +
         glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    op = gzip.open if f.endswith(".gz") else open
    with op(f, "rt") as fh:
        rows = list(csv.DictReader(fh))
    out = []
    for r in rows:
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("<")[0]))
    out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--linearizations", type=int, default=8)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ks = load(a.trace)
    lin = [i for i, k in enumerate(ks) if k[2] == "k_linearize_own"]
    start_i = lin[a.linearizations]
    seg = ks[start_i:]
    t0 = seg[0][0]
    t1 = max(e for _, e, _ in seg)
    busy = 0
    cur_s, cur_e = seg[0][0], seg[0][1]
    gaps = []   # (length ns, family before the gap, family after)
    last_name = seg[0][2]
    for s, e, n in seg[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, last_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            last_name = n
    busy += cur_e - cur_s
    span = t1 - t0
    idle = span - busy
    hist = collections.Counter()
    after = collections.defaultdict(lambda: [0, 0])
    for g, before, nxt in gaps:
        b = "<2us" if g < 2000 else "2-10us" if g < 10000 else "10-100us" if g < 100000 else ">=100us"
        hist[b] += g
        after[before][0] += 1
        after[before][1] += g
    res = {"span_ms": span / 1e6, "busy_ms": busy / 1e6, "idle_ms": idle / 1e6, "kernels": len(seg),
           "idle_by_gap_size_ms": {k: v / 1e6 for k, v in sorted(hist.items())},
           "idle_after_family_ms": {k: {"gaps": v[0], "ms": v[1] / 1e6}
                                    for k, v in sorted(after.items(), key=lambda kv: -kv[1][1])[:12]}}
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
