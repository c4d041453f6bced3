"""Turn a gpurun_out/prof tree (scripts/gpu_profile.sh) into committed profiles/ artifacts.

    python scripts/summarize_profile.py <tag> [gpurun_out/prof]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats of the
default C3 bench step), profiles/<tag>_pmc.json (per-launch FETCH_SIZE /
WRITE_SIZE medians) and updates profiles/pmc_traffic.json, which bench.py reads
for roofline.traffic.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md
§7: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
(The kernels here load 8 B per lane, which the guide calls uncalibrated; the
doubled figure is therefore an upper estimate.)
"""
import csv
import gzip
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
    per = {}
    for r in rows:
        per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: {"launches": len(v), "median_kib": statistics.median(v), "mean_kib": sum(v) / len(v)}
            for k, v in per.items()}


def short(name):
    """'void pgo::k_panel_syrk<...>(pgo::CholDev, ...)' -> 'k_panel_syrk'."""
    base = name.split("(")[0].split("<")[0]
    return base.split("::")[-1].split(" ")[-1]


def find(d, suffix):
    for base, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(base, f)
    return None


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = find(os.path.join(src, "trace"), "kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch = counters(find(os.path.join(src, "pmc_FETCH_SIZE"), "counter_collection.csv.gz"))
    write = counters(find(os.path.join(src, "pmc_WRITE_SIZE"), "counter_collection.csv.gz"))
    summary = {"tag": tag, "config": "C3", "formula": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024",
               "note": "per launch: mean over the launches of the first linearisation (launch sizes vary "
                       "for the Cholesky kernels), median also given", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, {}), write.get(k, {})
        ent = {"launches": f.get("launches"), "FETCH_SIZE_kib_mean": f.get("mean_kib"),
               "WRITE_SIZE_kib_mean": w.get("mean_kib"), "FETCH_SIZE_kib_median": f.get("median_kib"),
               "WRITE_SIZE_kib_median": w.get("median_kib")}
        ok = f and w
        ent["hbm_bytes_per_launch"] = (2 * f["mean_kib"] + w["mean_kib"]) * 1024 if ok else None
        ent["hbm_bytes_per_launch_median"] = (2 * f["median_kib"] + w["median_kib"]) * 1024 if ok else None
        summary["kernels"][short(k)] = ent
    with open(os.path.join(out, f"{tag}_pmc.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    traffic_path = os.path.join(out, "pmc_traffic.json")
    traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
    ent = traffic.get("C3", {})
    ent["source"] = f"{tag}_pmc.json"
    ent["lanes"] = 1   # the PMC passes run one lambda lane (gpu_profile.sh --lanes 1)
    for k in sorted(summary["kernels"]):
        v = summary["kernels"][k].get("hbm_bytes_per_launch")
        if v is not None:
            ent[f"{k}_bytes_per_launch"] = v
    # the one-lane launches' algorithmic flops (the trace run's own table), so
    # bench.py can scale the bytes to its launches' lane mix
    tb = os.path.join(src, "trace_bench.log")
    if os.path.exists(tb):
        lines = [l for l in open(tb) if l.startswith("{")]
        if lines:
            fams = (json.loads(lines[-1]).get("roofline") or {}).get("families") or {}
            for k, f in fams.items():
                if f.get("flops_per_launch"):
                    ent[f"{k}_flops_per_launch"] = f["flops_per_launch"]
    traffic["C3"] = ent
    with open(traffic_path, "w") as fh:
        json.dump(traffic, fh, indent=1)
    for logname in ("trace_bench.log",):
        p = os.path.join(src, logname)
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                with open(os.path.join(out, f"{tag}_profiled_bench.json"), "w") as fh:
                    fh.write(lines[-1])
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
