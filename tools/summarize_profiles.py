"""Copy one profile_round.sh output set into profiles/ and summarise it.

    python tools/summarize_profiles.py r01 [kernel]

Writes profiles/<tag>_bench.json (the bench line), <tag>_bench_kernel_stats.csv,
<tag>_bench_kernel_trace.csv, <tag>_pmc_fetch_size.csv, <tag>_pmc_write_size.csv
and profiles/pmc_summary.json (HBM bytes per launch of the hot kernel, which
bench.py reports as roofline.traffic).  FETCH_SIZE is doubled for gfx950's
half-count of wide reads (MI355X_MICROARCH.md, HBM section).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(pattern):
    hits = sorted(glob.glob(pattern), key=os.path.getmtime)
    if not hits:
        raise SystemExit("missing: " + pattern)
    return hits[-1]  # the newest run


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    kernel = sys.argv[2] if len(sys.argv) > 2 else "k_render<0, false, "  # EXACT, no stats, either stack
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, tag + "_bench.json"))
    shutil.copy(one(os.path.join(src, "trace", "*", "*_kernel_stats.csv")), os.path.join(dst, tag + "_bench_kernel_stats.csv"))
    shutil.copy(one(os.path.join(src, "trace", "*", "*_kernel_trace.csv")), os.path.join(dst, tag + "_bench_kernel_trace.csv"))
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = one(os.path.join(src, "pmc_" + c, "*", "*_counter_collection.csv"))
        shutil.copy(f, os.path.join(dst, "%s_pmc_%s.csv" % (tag, c.lower())))
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                if kernel in r["Kernel_Name"] and r["Counter_Name"] == c]
        per[c] = (sum(vals) / len(vals), len(vals))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, tag + "_bench_kernel_stats.csv")))}
    avg_ns = next(float(v["AverageNs"]) for k, v in stats.items() if kernel in k)
    bench = json.loads(open(os.path.join(dst, tag + "_bench.json")).read().strip().splitlines()[-1])
    rd = per["FETCH_SIZE"][0] * 1024 * 2
    wr = per["WRITE_SIZE"][0] * 1024
    out = {"workload": "bench.py --no-cpu --steps %d --warmup %d (%s), %d frames per launch in blocks of %d" % (
               bench["steps"], bench["steps"], bench["config"]["workload"], bench["steps"],
               bench["config"].get("frames_per_block", 16)),
           "kernel": kernel, "launches_averaged": per["FETCH_SIZE"][1],
           "FETCH_SIZE_kB_per_launch": per["FETCH_SIZE"][0], "WRITE_SIZE_kB_per_launch": per["WRITE_SIZE"][0],
           "hbm_read_bytes_per_launch_corrected": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr,
           "rocprof_avg_launch_ms": avg_ns / 1e6,
           "bench_avg_launch_ms": (bench.get("roofline") or {}).get("avg_launch_ms"),
           "note": "separate --pmc passes (MI355X_MICROARCH.md HBM section): FETCH_SIZE doubled for the gfx950 "
                   "half-count; this kernel's reads are 64-B gathers, for which the doubling is uncalibrated "
                   "(raw read bytes = half). Counts include Infinity-Cache hits.",
           "source": ["profiles/%s_pmc_fetch_size.csv" % tag, "profiles/%s_pmc_write_size.csv" % tag,
                      "profiles/%s_bench_kernel_stats.csv" % tag]}
    out["frames_per_launch"] = bench["steps"]
    wl = bench["config"]["workload"].split(":")[0]
    path = os.path.join(dst, "pmc_summary.json")
    try:
        allw = json.load(open(path))
        if "kernel" in allw:  # the old single-workload layout
            allw = {}
    except (OSError, ValueError):
        allw = {}
    allw[wl] = out
    with open(path, "w") as fh:
        json.dump(allw, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
