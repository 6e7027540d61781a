"""rocprofv3 evidence for bench.py's roofline, on the bench's own command.

On the GPU box (one gpurun call; every pass is its own process under its own
time limit, counters in separate --pmc passes as MI355X_MICROARCH.md asks):

    python tools/profile.py run <tag> [bench args ...]     # e.g. r02 --steps 20 --warmup 5

  gpurun_out/prof_<tag>/bench.json          the bench line of the exact command
  gpurun_out/prof_<tag>/trace/              --kernel-trace --stats of the same command (--no-cpu)
  gpurun_out/prof_<tag>/pmc_<pass>/         one --pmc pass each (PASSES below)
  gpurun_out/prof_<tag>/calib_<pass>/       FETCH_SIZE / WRITE_SIZE of the gather-calibration
                                            kernel (mcpt_gather_probe, 64- and 128-B records)

Back here:

    python tools/profile.py summarize <tag>
    python tools/profile.py refit            # the TD floor model over every committed profile

copies the CSVs to profiles/<tag>_*.csv (trimmed to the timed dispatch's rows,
tools/trim_profiles.py) and writes profiles/<tag>_summary.json
plus the entry of profiles/pmc_summary.json that bench.py reads (keyed by
workload and frames per call).  The timed launch is the LAST dispatch of the
bench's non-counting k_render instantiation (bench order: schedule tuning,
warmup, timed call, then the counting replay with a different
instantiation); its per-dispatch counters are the ones summarised.
"""
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# one rocprofv3 --pmc pass each (block limits: 8 SQ, 4 TCC with FETCH_SIZE=3
# and WRITE_SIZE=2, 4 TCP, 2 GRBM)
PASSES = {
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
    "sq": ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
           "SQ_WAIT_ANY", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "GRBM_GUI_ACTIVE"],
    "sq2": ["SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
            "SQ_WAIT_INST_ANY", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_VMEM_WR", "GRBM_GUI_ACTIVE"],
    "cache": ["TCC_HIT_sum", "TCC_MISS_sum", "TCP_TCC_READ_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum"],
    "lat": ["TCP_TCP_LATENCY_sum", "TCP_TCC_READ_REQ_LATENCY_sum", "TA_TA_BUSY_sum", "TD_TD_BUSY_sum"],
    "derived": ["VALUBusy", "VALUUtilization"],
}
HBM_PEAK_GBS = 8000.0
N_CU_DEFAULT = 256  # MI355X; summarize() reads the profiled device's count (device.json)


def sh(cmd, log, limit):
    with open(log, "w") as fh:
        r = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, stdout=fh, stderr=subprocess.STDOUT,
                           cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        print("FAILED (%d): %s\n%s" % (r.returncode, " ".join(cmd), open(log).read()[-3000:]), flush=True)
        sys.exit(1)


def run(tag, args):
    out = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    os.makedirs(out, exist_ok=True)
    bench = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    print("bench:", " ".join(args), flush=True)
    with open(os.path.join(out, "bench.json"), "w") as fh:
        r = subprocess.run(["timeout", "-k", "10", "400"] + bench, stdout=fh, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        print(r.stderr[-3000:])
        sys.exit(1)
    line = open(os.path.join(out, "bench.json")).read().strip()
    print(line[-600:], flush=True)
    # the same command with the schedule the bench line's tuning picked, so
    # every pass profiles the same kernel instantiation
    cfg = json.loads(line.splitlines()[-1])["config"]
    quiet = bench + ["--no-cpu", "--no-cache-off", "--schedule", cfg["schedule"], "--shade-threshold", str(cfg.get("shade_threshold", 32)),
                     "--fetch-threshold", str(cfg.get("fetch_threshold", 1)),
                     "--block-entries", str(cfg.get("block_entries", 8))]
    if cfg.get("last_block_frames"):  # 0: the auto rule, which the pinned command keeps (it does not tune)
        quiet += ["--last-block-frames", str(cfg["last_block_frames"])]
    if "tile_order" in cfg:
        quiet += ["--tile-order", str({"dearest first (costliest pixel)": 0, "image": 1,
                                       "dearest first (summed)": 2}[cfg["tile_order"]])]
    if "--quantized" in args:  # the search-tree format the command forced
        quiet += ["--quantized", args[args.index("--quantized") + 1]]
    sh(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", os.path.join(out, "trace"), "--"]
       + quiet, os.path.join(out, "trace.log"), 400)
    print("trace done", flush=True)
    # the CU count the busy ratios divide by, read from the device
    sh([sys.executable, "-c", "import json, torch; p = torch.cuda.get_device_properties(0); "
        "json.dump({'cus': p.multi_processor_count, 'name': p.name}, open(%r, 'w'))" % os.path.join(out, "device.json")],
       os.path.join(out, "device.log"), 120)
    for name, ctrs in PASSES.items():
        sh(["rocprofv3", "--pmc"] + ctrs + ["--output-format", "csv", "-d", os.path.join(out, "pmc_" + name), "--"]
           + quiet, os.path.join(out, "pmc_%s.log" % name), 300)
        print("pmc", name, "done", flush=True)
    calib = [sys.executable, os.path.join(ROOT, "tools", "profile.py"), "calib"]
    for name in ("fetch", "write"):
        sh(["rocprofv3", "--pmc"] + PASSES[name] + ["--output-format", "csv", "-d", os.path.join(out, "calib_" + name),
                                                    "--"] + calib, os.path.join(out, "calib_%s.log" % name), 200)
    print("calibration done", flush=True)
    # the TD model: cycles per gather instruction against the
    # distinct lines it touches, by the committed microbenchmark, timed alone
    # and then once under the counters the model multiplies (lines per
    # instruction checked against TCP_TOTAL_CACHE_ACCESSES)
    mb = os.path.join(ROOT, "tools", "mb", "td_lanes")
    sh([mb, "--json"], os.path.join(out, "tdcal.jsonl"), 120)
    sh(["rocprofv3", "--pmc", "SQ_INSTS_VMEM_RD", "TCP_TOTAL_CACHE_ACCESSES_sum", "TD_TD_BUSY_sum", "GRBM_GUI_ACTIVE",
        "--output-format", "csv", "-d", os.path.join(out, "tdcal_pmc"), "--", mb], os.path.join(out, "tdcal_pmc.log"), 120)
    print("TD calibration done", flush=True)


def calib():
    """The calibration kernel alone (run under rocprofv3 by `run`)."""
    sys.path.insert(0, ROOT)
    from montecarlopathtracing_amd import render as R
    rnd = R.Renderer(0)
    for rec in (128, 64):
        ms = rnd.gather_probe(rec, 1 << 31)
        print("gather_probe %d-B records, 2 GiB table: %.3f ms = %.1f GB/s" % (rec, ms, (1 << 31) / ms / 1e6))


def newest(pattern):
    hits = sorted(glob.glob(pattern), key=os.path.getmtime)
    if not hits:
        raise SystemExit("missing: " + pattern)
    return hits[-1]


def dispatches(path, name_re):
    """{dispatch_id: {counter: value, "kernel": name}} for kernels matching name_re."""
    out = {}
    for r in csv.DictReader(open(path)):
        if re.search(name_re, r["Kernel_Name"]):
            d = out.setdefault(int(r["Dispatch_Id"]), {"kernel": r["Kernel_Name"]})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    return out


def summarize(tag):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    bench_line = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    bench = json.loads(bench_line)
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, tag + "_bench.json"))
    stats_csv = newest(os.path.join(src, "trace", "*", "*_kernel_stats.csv"))
    trace_csv = newest(os.path.join(src, "trace", "*", "*_kernel_trace.csv"))
    shutil.copy(stats_csv, os.path.join(dst, tag + "_kernel_stats.csv"))
    shutil.copy(trace_csv, os.path.join(dst, tag + "_kernel_trace.csv"))
    sched = bench["config"]["schedule"]
    quant = "true" if bench["config"].get("search_tree_nodes", "").startswith("64") else "false"
    # the render instantiation (PRIM = false), not the primary-hit pass (PRIM = true)
    kname = r"k_render<0, false, (false|true), %s, %s, false, (false|true)(, [a-z0-9]+)?>" % (
        "true" if sched == "paired" else "false", quant)
    trace = [r for r in csv.DictReader(open(trace_csv)) if re.search(kname, r["Kernel_Name"])]
    timed = trace[-1]
    timed_ms = (int(timed["End_Timestamp"]) - int(timed["Start_Timestamp"])) / 1e6
    same = [r for r in trace if r["Kernel_Name"] == timed["Kernel_Name"]]
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
    st = stats.get(timed["Kernel_Name"], {})
    ctr = {}
    for name in PASSES:
        f = newest(os.path.join(src, "pmc_" + name, "*", "*_counter_collection.csv"))
        shutil.copy(f, os.path.join(dst, "%s_pmc_%s.csv" % (tag, name)))
        ds = dispatches(f, kname)
        last = ds[max(ds)]  # the timed launch: the last dispatch of the instantiation
        ctr.update({k: v for k, v in last.items() if k != "kernel"})
    cal = {}
    for name in ("fetch", "write"):
        f = newest(os.path.join(src, "calib_" + name, "*", "*_counter_collection.csv"))
        shutil.copy(f, os.path.join(dst, "%s_calib_%s.csv" % (tag, name)))
        ds = dispatches(f, r"k_gather_probe")
        ids = sorted(ds)  # run order: 128-B records, then 64-B
        c = PASSES[name][0]
        cal[name] = {"128": ds[ids[0]][c] * 1024.0, "64": ds[ids[1]][c] * 1024.0}
    known = float(1 << 31)
    # FETCH_SIZE scale for this kernel's gathers: known bytes / counted bytes
    # of the calibration kernel, record sizes weighted as k_render reads them
    # (128-B nodes and 64-B triangles per segment, from the bench's counters)
    r = bench.get("roofline") or {}
    n_node, n_tri = r.get("kernel_node_fetches_per_seg", 7.16), r.get("kernel_tri_tests_per_seg", 2.97)
    s128, s64 = known / cal["fetch"]["128"], known / cal["fetch"]["64"]
    w128 = 128.0 * n_node / (128.0 * n_node + 64.0 * n_tri)
    fetch_scale = w128 * s128 + (1 - w128) * s64
    rd_raw = ctr["FETCH_SIZE"] * 1024.0
    wr = ctr["WRITE_SIZE"] * 1024.0
    rd = rd_raw * fetch_scale
    secs = timed_ms / 1e3
    try:
        N_CU = int(json.load(open(os.path.join(src, "device.json")))["cus"])
    except (OSError, ValueError, KeyError):
        N_CU = N_CU_DEFAULT
    grbm = ctr["GRBM_GUI_ACTIVE"]  # summed over the 8 XCDs (MI355X_MICROARCH.md)
    cycles = grbm / 8.0
    l2_req = ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"]
    td = td_model(src, ctr, N_CU, cycles)
    summ = {
        "tag": tag, "command": "python3 bench.py " + " ".join(bench_args_of(bench)),
        "workload": bench["config"]["workload"], "steps": bench["steps"], "warmup": bench["warmup"],
        "frames_per_block": bench["config"].get("frames_per_block"),
        "kernel": timed["Kernel_Name"], "timed_dispatch_id": int(timed["Dispatch_Id"]),
        "timed_launch_ms_rocprof": round(timed_ms, 4),
        "bench_avg_launch_ms": r.get("avg_launch_ms"),
        "rocprof_stats_average_ms_all_dispatches_of_kernel": round(float(st.get("AverageNs", 0)) / 1e6, 4),
        "dispatches_of_kernel": len(same),
        "FETCH_SIZE_bytes_raw": rd_raw, "WRITE_SIZE_bytes": wr,
        "fetch_scale_calibrated": round(fetch_scale, 4),
        "calibration": {"known_bytes": known, "FETCH_SIZE_bytes_128B_records": cal["fetch"]["128"],
                        "FETCH_SIZE_bytes_64B_records": cal["fetch"]["64"],
                        "WRITE_SIZE_bytes_128B_records": cal["write"]["128"],
                        "WRITE_SIZE_bytes_64B_records": cal["write"]["64"],
                        "scale_128": round(s128, 4), "scale_64": round(s64, 4), "weight_128": round(w128, 4)},
        "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes": rd + wr,
        "hbm_GBps": round((rd + wr) / secs / 1e9, 2), "hbm_frac": round((rd + wr) / secs / 1e9 / HBM_PEAK_GBS, 5),
        "kernel_cycles": cycles, "clock_GHz": round(cycles / secs / 1e9, 3), "cus": N_CU,
        "valu_busy": round(ctr["SQ_ACTIVE_INST_VALU"] / (N_CU * cycles), 4),
        "valu_busy_rocprof_derived": round(ctr.get("VALUBusy", float("nan")) / 100.0, 4),
        "valu_utilization_lanes": round(ctr.get("VALUUtilization", float("nan")) / 100.0, 4),
        "wave_issue_any_per_wave_cycle": round(ctr["SQ_ACTIVE_INST_ANY"] / ctr["SQ_WAVE_CYCLES"], 4),
        "wave_wait_any_per_wave_cycle": round(ctr["SQ_WAIT_ANY"] / ctr["SQ_WAVE_CYCLES"], 4),
        "waves_per_simd_avg": round(ctr["SQ_WAVE_CYCLES"] / (N_CU * 4 * cycles / 4.0), 3),
        "valu_insts": ctr["SQ_INSTS_VALU"], "vmem_rd_insts": ctr["SQ_INSTS_VMEM_RD"],
        "salu_insts": ctr.get("SQ_INSTS_SALU"), "lds_insts": ctr.get("SQ_INSTS_LDS"),
        "l1_accesses": ctr["TCP_TOTAL_CACHE_ACCESSES_sum"], "l1_to_l2_reads": ctr["TCP_TCC_READ_REQ_sum"],
        "l1_hit_rate": round(1 - ctr["TCP_TCC_READ_REQ_sum"] / max(ctr["TCP_TOTAL_CACHE_ACCESSES_sum"], 1), 4),
        "l2_requests": l2_req, "l2_hit_rate": round(ctr["TCC_HIT_sum"] / max(l2_req, 1), 4),
        "l2_hit_GBps_128B_lines": round(ctr["TCC_HIT_sum"] * 128.0 / secs / 1e9, 1),
        "gather_latency_cycles_per_vmem_rd": round(ctr["TCP_TCP_LATENCY_sum"] / max(ctr["SQ_INSTS_VMEM_RD"], 1), 1),
        "ta_busy_sum": ctr.get("TA_TA_BUSY_sum"), "td_busy_sum": ctr.get("TD_TD_BUSY_sum"),
        # vector-memory address (TA) and data-return (TD) units: busy cycles per CU per kernel cycle
        "ta_busy": round(ctr.get("TA_TA_BUSY_sum", float("nan")) / (N_CU * cycles), 4),
        "td_busy": round(ctr.get("TD_TD_BUSY_sum", float("nan")) / (N_CU * cycles), 4),
        # the bench line's roofline recomputed with THIS run's counters (the bench
        # line itself ran before them and carries the previous pmc_summary.json)
        "roofline_this_run": {
            "traffic": rd + wr, "avg_launch_ms": r.get("avg_launch_ms"),
            "achieved": round((rd + wr) / (r["avg_launch_ms"] / 1e3) / 1e9, 2) if r.get("avg_launch_ms") else None,
            "frac": round((rd + wr) / (r["avg_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 5) if r.get("avg_launch_ms") else None,
            "valu_busy": round(ctr["SQ_ACTIVE_INST_VALU"] / (N_CU * cycles), 4),
            "issue_frac": round(ctr["SQ_ACTIVE_INST_VALU"] / (N_CU * cycles) * ctr.get("VALUUtilization", float("nan")) / 100.0, 4),
            "td_busy": round(ctr.get("TD_TD_BUSY_sum", float("nan")) / (N_CU * cycles), 4)},
        "td_model": td,
        "counters_timed_dispatch": ctr,
        "sources": ["profiles/%s_%s.csv" % (tag, x) for x in
                    ["kernel_stats", "kernel_trace"] + ["pmc_" + n for n in PASSES] + ["calib_fetch", "calib_write"]],
        "note": "counters of the timed launch only (last dispatch of the bench's non-counting k_render); "
                "GRBM_GUI_ACTIVE is summed over the 8 XCDs (cycles = /8); SQ_* cycle counters are quad-cycles; "
                "valu_busy = SQ_ACTIVE_INST_VALU / (CUs x cycles) (rocprofv3's VALUBusy definition; it can read ~1 % "
                "over 1 on a VALU-saturated kernel, as rocprofv3's own VALUBusy does); issue_frac = valu_busy x "
                "VALUUtilization (lane-weighted); "
                "hbm bytes = FETCH_SIZE x calibrated scale + WRITE_SIZE (memory-side: Infinity-Cache hits included)",
    }
    with open(os.path.join(dst, tag + "_summary.json"), "w") as fh:
        json.dump(summ, fh, indent=1)
    key = "%s@%d" % (bench["config"]["workload"].split(":")[0], bench["steps"])
    path = os.path.join(dst, "pmc_summary.json")
    try:
        allw = json.load(open(path))
    except (OSError, ValueError):
        allw = {}
    allw = {k: v for k, v in allw.items() if "@" in k}  # drop the round-1 layout
    allw[key] = {"hbm_bytes_per_launch": rd + wr, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                 "fetch_scale_calibrated": summ["fetch_scale_calibrated"], "valu_busy": summ["valu_busy"],
                 "valu_utilization_lanes": summ["valu_utilization_lanes"],
                 "ta_busy": summ["ta_busy"], "td_busy": summ["td_busy"],
                 "wave_wait_any_per_wave_cycle": summ["wave_wait_any_per_wave_cycle"],
                 "l2_hit_rate": summ["l2_hit_rate"], "l1_hit_rate": summ["l1_hit_rate"],
                 "l2_hit_GBps_128B_lines": summ["l2_hit_GBps_128B_lines"],
                 "gather_latency_cycles_per_vmem_rd": summ["gather_latency_cycles_per_vmem_rd"],
                 "timed_launch_ms_rocprof": summ["timed_launch_ms_rocprof"], "frames_per_block": summ["frames_per_block"],
                 "kernel_cycles": cycles, "clock_GHz": summ["clock_GHz"],
                 "source": "profiles/%s_summary.json" % tag}
    if td:
        allw[key]["td_model"] = {k: td[k] for k in ("a_cycles_per_inst", "b_cycles_per_line", "vmem_rd_insts",
                                                    "l1_accesses", "floor_cycles_per_cu", "model_frac", "td_busy",
                                                    "td_busy_saturated_microbench", "busy_frac")}
    with open(path, "w") as fh:
        json.dump(allw, fh, indent=1, sort_keys=True)
    # keep only the rows the summary is computed from (tools/trim_profiles.py):
    # the timed dispatch of each --pmc pass, the render kernels of the trace
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import trim_profiles
    trim_profiles.main(sorted(glob.glob(os.path.join(dst, tag + "_*.csv"))))
    refit()  # the TD floor model over every committed profile, this one included
    print(json.dumps(summ, indent=1))


def td_model(src, ctr, n_cu, cycles):
    """The TD (vector-memory data path) bound of the timed launch, two ways.
    Measured: TD_TD_BUSY per CU per cycle of the launch, against the same
    counter on the microbenchmark's saturating pattern (tools/mb/td_lanes.hip
    mode 0, 64 lanes each gathering their own 128-B record, 16 waves per CU:
    k_render's node-step shape) -> busy_frac.  Modelled: the microbenchmark's
    cycles per wave gather instruction per CU against the lines it touches,
    fitted on its mode-0 points as cycles = a + b * lines; the launch's floor
    is (a * SQ_INSTS_VMEM_RD + b * TCP_TOTAL_CACHE_ACCESSES) / CUs cycles and
    model_frac = floor / kernel cycles.  None when the calibration was not
    run (profiles before round 4)."""
    path = os.path.join(src, "tdcal.jsonl")
    if not os.path.exists(path):
        return None
    import numpy as np
    tag = os.path.basename(src).replace("prof_", "")
    pts = [json.loads(x) for x in open(path) if x.startswith("{")]
    m0 = [p for p in pts if p["mode"] == 0]
    A = np.array([[1.0, p["lines"]] for p in m0])
    y = np.array([p["cycles_per_inst"] for p in m0])
    (a, b), *_ = np.linalg.lstsq(A, y, rcond=None)
    resid = y - A @ np.array([a, b])
    shutil.copy(path, os.path.join(ROOT, "profiles", tag + "_tdcal.jsonl"))
    # the counters' view of the same patterns (accesses per instruction = the
    # designed lines; TD busy of the saturating pattern)
    lines_ctr, sat = None, None
    try:
        f = newest(os.path.join(src, "tdcal_pmc", "*", "*_counter_collection.csv"))
        shutil.copy(f, os.path.join(ROOT, "profiles", tag + "_tdcal_pmc.csv"))
        ds = dispatches(f, r"^k\(|k\(float")
        ids = sorted(ds)[1::2]  # each pattern: a warm dispatch, then the timed one
        lines_ctr = [round(ds[i]["TCP_TOTAL_CACHE_ACCESSES_sum"] / max(ds[i]["SQ_INSTS_VMEM_RD"], 1), 2) for i in ids]
        d0 = ds[ids[0]]  # mode 0, 64 active lanes
        sat = d0["TD_TD_BUSY_sum"] / (n_cu * d0["GRBM_GUI_ACTIVE"] / 8.0)
    except SystemExit:
        pass
    vm, acc = ctr["SQ_INSTS_VMEM_RD"], ctr["TCP_TOTAL_CACHE_ACCESSES_sum"]
    floor = (a * vm + b * acc) / n_cu
    busy = ctr["TD_TD_BUSY_sum"] / (n_cu * cycles)
    return {"a_cycles_per_inst": round(float(a), 3), "b_cycles_per_line": round(float(b), 4),
            "fit_max_abs_resid_cycles": round(float(np.abs(resid).max()), 2),
            "points": [{k: p[k] for k in ("mode", "active", "lines", "cycles_per_inst")} for p in pts],
            "counter_lines_per_inst": lines_ctr,
            "vmem_rd_insts": vm, "l1_accesses": acc, "l1_accesses_per_vmem_rd": round(acc / max(vm, 1), 2),
            "floor_cycles_per_cu": round(floor, 1), "kernel_cycles": cycles, "model_frac": round(floor / cycles, 4),
            "td_busy": round(busy, 4), "td_busy_saturated_microbench": None if sat is None else round(sat, 4),
            "busy_frac": None if not sat else round(busy / sat, 4),
            "note": "busy_frac = the launch's TD busy / the saturating microbenchmark's (measured); model_frac = "
                    "(a x SQ_INSTS_VMEM_RD + b x TCP_TOTAL_CACHE_ACCESSES_sum) / CUs / kernel cycles with a, b "
                    "from the microbenchmark's own-line-per-lane points; a holds for any active-lane count (a "
                    "1-lane gather costs ~18 cycles, a 64-lane one on 64 lines ~65), so SIMT efficiency moves it"}


B_LINE_MICROBENCH = 0.7435  # tools/mb/td_lanes.hip: TD cycles per L1 line a gather touches (r04a_tdcal)


def refit():
    """The TD floor model, fitted on every committed profile (VERDICT r4 next
    3): TD_TD_BUSY_sum = a x SQ_INSTS_VMEM_RD + b x L1-hit line accesses +
    c x TCP_TCC_READ_REQ_sum (L1 misses), non-negative least squares over the
    timed launches of profiles/*_summary.json (C2-C5, rounds 2-5).  Writes
    profiles/td_floor_fit.json (coefficients, each profile's modelled / measured
    busy) and adds each pmc_summary.json entry's fitted floor ("td_fit"):
    floor_cycles_per_cu, model_frac = floor / kernel cycles, the per-instruction
    term's share of it, and TD busy per cycle (<= 1 by construction)."""
    import numpy as np
    from scipy.optimize import nnls
    dst = os.path.join(ROOT, "profiles")
    rows = []
    for f in sorted(glob.glob(os.path.join(dst, "*_summary.json"))):
        s = json.load(open(f))
        c = s.get("counters_timed_dispatch", {})
        if not all(k in c for k in ("TD_TD_BUSY_sum", "TCP_TCC_READ_REQ_sum", "SQ_INSTS_VMEM_RD",
                                    "TCP_TOTAL_CACHE_ACCESSES_sum")):
            continue
        rows.append((os.path.basename(f)[:-len("_summary.json")], s["workload"].split(":")[0], c))
    X = np.array([[c["SQ_INSTS_VMEM_RD"], c["TCP_TOTAL_CACHE_ACCESSES_sum"] - c["TCP_TCC_READ_REQ_sum"],
                   c["TCP_TCC_READ_REQ_sum"]] for _, _, c in rows])
    y = np.array([c["TD_TD_BUSY_sum"] for _, _, c in rows])
    (a, b, cm), _ = nnls(X, y)
    ratio = {t: round(float(p / m), 4) for (t, _, _), p, m in zip(rows, X @ np.array([a, b, cm]), y)}
    # the free fit is degenerate: across these profiles (one kernel family)
    # gather instructions and line accesses move together (collinear), and NNLS
    # puts the line term at b = 0.  The TD microbenchmark measures the per-line
    # cost directly (tools/mb/td_lanes.hip: 0.74 cycle per line, 64 lines 65.0
    # cycles, 1 line 18.0), so the second fit holds b there and fits a and c
    b_mb = B_LINE_MICROBENCH
    (a2, c2), _ = nnls(X[:, [0, 2]], y - b_mb * X[:, 1])
    ratio2 = {t: round(float(p / m), 4) for (t, _, _), p, m in zip(rows, X @ np.array([a2, b_mb, c2]), y)}
    corr = float(np.corrcoef(X[:, 0], X[:, 1])[0, 1])
    by_wl = {}
    for (t, wl, _), r in zip(rows, ratio.values()):
        by_wl.setdefault(wl, []).append(r)
    fit = {"a_cycles_per_gather_inst": round(float(a), 4), "b_cycles_per_l1_hit_line": round(float(b), 4),
           "c_cycles_per_l2_request": round(float(cm), 4), "profiles": len(rows),
           "modelled_over_measured_busy": ratio,
           "corr_gather_insts_vs_l1_hit_lines": round(corr, 4),
           "b_fixed": {"a_cycles_per_gather_inst": round(float(a2), 4), "b_cycles_per_l1_hit_line": b_mb,
                       "c_cycles_per_l2_request": round(float(c2), 4), "modelled_over_measured_busy": ratio2,
                       "note": "b held at the microbenchmark's per-line cost; a, c by NNLS on the rest"},
           "range_by_workload": {k: [min(v), max(v)] for k, v in sorted(by_wl.items())},
           "note": "TD_TD_BUSY_sum (busy cycles summed over CUs) = a x SQ_INSTS_VMEM_RD + b x (TCP_TOTAL_CACHE_ACCESSES_sum "
                   "- TCP_TCC_READ_REQ_sum) + c x TCP_TCC_READ_REQ_sum, non-negative least squares over the timed launch of "
                   "every committed profile; the floor of a launch = that sum / CUs, model_frac = floor / kernel cycles"}
    with open(os.path.join(dst, "td_floor_fit.json"), "w") as fh:
        json.dump(fit, fh, indent=1, sort_keys=True)
    path = os.path.join(dst, "pmc_summary.json")
    allw = json.load(open(path))
    for key, e in allw.items():
        src = os.path.join(ROOT, e.get("source", ""))
        if not os.path.exists(src):
            continue
        s = json.load(open(src))
        c = s.get("counters_timed_dispatch", {})
        if "TCP_TCC_READ_REQ_sum" not in c or "TD_TD_BUSY_sum" not in c:
            continue
        n_cu, cyc = s.get("cus", N_CU_DEFAULT), s["kernel_cycles"]
        vm, acc, l2 = c["SQ_INSTS_VMEM_RD"], c["TCP_TOTAL_CACHE_ACCESSES_sum"], c["TCP_TCC_READ_REQ_sum"]
        floor = a * vm + b * (acc - l2) + cm * l2
        floor2 = a2 * vm + b_mb * (acc - l2) + c2 * l2
        e["td_fit"] = {"floor_cycles_per_cu": round(float(floor / n_cu), 1), "kernel_cycles": cyc,
                       "model_frac": round(float(floor / n_cu / cyc), 4),
                       "inst_term_share": round(float(a * vm / max(floor, 1.0)), 4),
                       "model_frac_b_fixed": round(float(floor2 / n_cu / cyc), 4),
                       "inst_term_share_b_fixed": round(float(a2 * vm / max(floor2, 1.0)), 4),
                       "td_busy_per_cycle": round(c["TD_TD_BUSY_sum"] / (n_cu * cyc), 4),
                       "vmem_rd_insts": vm, "l1_accesses": acc, "l2_requests": l2,
                       "l1_lines_per_vmem_rd_inst": round(acc / max(vm, 1), 2), "fit": "profiles/td_floor_fit.json"}
    with open(path, "w") as fh:
        json.dump(allw, fh, indent=1, sort_keys=True)
    print(json.dumps(fit, indent=1))


def bench_args_of(b):
    return ["--gpus", str(b["n_gpus"]), "--steps", str(b["steps"]), "--warmup", str(b["warmup"])] + (
        [] if b["config"]["workload"].startswith("C2") else ["--workload", b["config"]["workload"].split(":")[0]])


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:])
    elif sys.argv[1] == "calib":
        calib()
    elif sys.argv[1] == "refit":
        refit()
    else:
        summarize(sys.argv[2])
