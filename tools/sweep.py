"""A/B sweeps of k_render launch-plan knobs (speed only; every setting gives
the same bits) on one GPU.

    python tools/sweep.py --workload C2 --frames 20 --reps 5 \
        --grid "queue_chunk=4,8,16 block_entries=8,16" [--fpl 0,5,20] [--schedule paired]

Every combination of the grid is timed `reps` times, interleaved round-robin
(so clock drift hits all alike), on the bench's own scene/state setup; prints
one line per combination: median kernel ms and nominal Msamples/s.  With
--stats the kernel's counters (segments, node/tri per segment, SIMT
efficiency per phase) of one extra call per combination are printed too.
"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402


def parse_grid(text):
    axes = []
    for part in (text or "").replace("+", " ").split():  # axes separated by spaces or '+
        k, vals = part.split("=")
        axes.append([(k, int(v)) for v in vals.split(",")])
    return [dict(c) for c in itertools.product(*axes)] if axes else [{}]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C2", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grid", default="")
    ap.add_argument("--fpl", default="0", help="comma list of frames_per_launch values (0 = auto)")
    ap.add_argument("--schedule", default="paired", choices=["single", "paired"])
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--calls", type=int, default=1, help="render the frames as this many back-to-back calls "
                    "(frames/calls each, stream-async, one sync at the end; the app's update() pattern): "
                    "wall-clock ms over all calls is reported as kernel_ms")
    ap.add_argument("--json", default=None, help="append result lines to this file")
    ap.add_argument("--drop", action="store_true", help="drop the primary-hit cache before every timed call "
                    "(the call then runs the primary-hit pass and builds its tile order, as bench.py's timed call does)")
    ap.add_argument("--stripes", default="1", help="comma list of stripe counts: rank 0's share of the image "
                    "(16-row stripes dealt round-robin) rendered alone = one rank of an N-GPU strong-scaled run")
    ap.add_argument("--all-ranks", action="store_true", help="with --stripes N: time every rank's share, not "
                    "only rank 0's; the job's time is the slowest share's (max over ranks)")
    ap.add_argument("--stripe-rows", type=int, default=16)
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    w, h, depth = wl["w"], wl["h"], wl["depth"]
    data, camj = bench.load_scene(a.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(0)
    dsc, _ = bench.upload_scene(rnd, data)
    dsc.schedule = L.SCHED_PAIRED if a.schedule == "paired" else L.SCHED_SINGLE
    st = rnd.new_state(w, h)
    combos = [(fpl, g, n, r) for n in (int(x) for x in a.stripes.split(",")) for fpl in (int(x) for x in a.fpl.split(","))
              for g in parse_grid(a.grid) for r in (range(n) if a.all_ranks else (0,))]
    times = {i: [] for i in range(len(combos))}
    ticks = {}
    fpb = {}
    prim = {}
    for i, (fpl, g, n, r) in enumerate(combos):  # warm every variant once
        rnd.set_tuning(**g)
        rnd.render_frames(dsc, cam, st, depth, 1 << 30, min(a.frames, 4), frames_per_launch=fpl, stripe_count=n, stripe_index=r, stripe_rows=a.stripe_rows)
    torch.cuda.synchronize()
    per_call = max(1, a.frames // max(a.calls, 1))
    for _ in range(a.reps):
        for i, (fpl, g, n, r) in enumerate(combos):
            rnd.set_tuning(**g)
            if a.calls > 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _c in range(a.calls):
                    rnd.render_frames(dsc, cam, st, depth, 1 << 30, per_call, frames_per_launch=fpl, stripe_count=n, stripe_index=r, stripe_rows=a.stripe_rows)
                torch.cuda.synchronize()
                s = rnd.stats()
                times[i].append((time.perf_counter() - t0) * 1e3)
            else:
                if a.drop:
                    rnd.drop_caches()
                rnd.render_frames(dsc, cam, st, depth, 1 << 30, a.frames, frames_per_launch=fpl, stripe_count=n, stripe_index=r, stripe_rows=a.stripe_rows)
                s = rnd.stats()
                times[i].append(s["kernel_ms"])
                if s.get("primary_cache") == 2:  # this call ran the primary-hit pass (part of kernel_ms)
                    prim.setdefault(i, []).append(s["primary_ms"])
            fpb[i] = s["frames_per_block"]
            if any(s["phase_ticks"]):  # an MCPT_PHASE_TIMING build (MCPT_LIB_OVERRIDE)
                ticks.setdefault(i, [0, 0, 0, 0])
                ticks[i] = [a + b for a, b in zip(ticks[i], s["phase_ticks"])]
    out = []
    for i, (fpl, g, n, r) in enumerate(combos):
        ts = sorted(times[i])
        med = ts[len(ts) // 2]
        rec = {"workload": a.workload, "frames": a.frames, "fpl": fpl, "fpb": fpb[i], "tuning": g,
               "kernel_ms_median": round(med, 3), "kernel_ms_min": round(ts[0], 3),
               "Msamples_s": round(w * h * a.frames * depth / (med / 1e3) / 1e6, 1)}
        if i in prim:
            ps = sorted(prim[i])
            rec["primary_ms_median"] = round(ps[len(ps) // 2], 4)
        if a.calls > 1:
            rec.update({"calls": a.calls, "frames_per_call": per_call, "wall_ms_median": rec.pop("kernel_ms_median"),
                        "ms_per_frame": round(med / (a.calls * per_call), 4)})
        if i in ticks:
            tot = float(sum(ticks[i]))
            rec["phase_frac_fetch_T_L_S"] = [round(t / tot, 4) for t in ticks[i]]
        if n > 1:  # one rank's share: the N-rank job's rate if every rank took as long
            rec.update({"stripes": n, "rank": r, "stripe_rows": a.stripe_rows, "Msamples_s": None,
                        "rank0_Msamples_s": round(w * h / n * a.frames * depth / (med / 1e3) / 1e6, 1),
                        "job_Msamples_s_if_balanced": round(w * h * a.frames * depth / (med / 1e3) / 1e6, 1)})
        if a.stats:
            rnd.set_tuning(**g)
            rnd.set_stats(True)
            rnd.render_frames(dsc, cam, st, depth, 1 << 30, a.frames, frames_per_launch=fpl, stripe_count=n, stripe_index=r, stripe_rows=a.stripe_rows)
            c = rnd.stats()
            rnd.set_stats(False)
            seg = max(c["segments"], 1)
            rec.update({"segments": c["segments"], "node_per_seg": round(c["node_visits"] / seg, 3),
                        "tri_per_seg": round(c["tri_tests"] / seg, 3),
                        "leaf_rejects_per_seg": round(c.get("leaf_rejects", 0) / seg, 3),
                        "simt_T": round(c["node_visits"] / (64.0 * max(c["wave_node_phases"], 1)), 3),
                        "simt_L": round(c["tri_tests"] / (64.0 * max(c["wave_leaf_phases"], 1)), 3),
                        "simt_S": round(seg / (64.0 * max(c["wave_shade_phases"], 1)), 3),
                        "waiting_frac": round(c["lane_waiting"] / (64.0 * max(c["wave_iterations"], 1)), 4),
                        "idle_frac": round(c["lane_idle"] / (64.0 * max(c["wave_iterations"], 1)), 4),
                        "iters_per_seg": round(c["wave_iterations"] * 64.0 / seg, 3),
                        "order_fallbacks": c["order_fallbacks"]})
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if a.all_ranks:  # the job: every rank's share at once, as slow as its slowest
        for (fpl, g) in {(c[0], json.dumps(c[1], sort_keys=True)) for c in combos}:
            for n in sorted({c[2] for c in combos}):
                ms = [r["kernel_ms_median"] for r, c in zip(out, combos) if c[0] == fpl and c[2] == n
                      and json.dumps(c[1], sort_keys=True) == g]
                if n < 2 or not ms:
                    continue
                job = {"workload": a.workload, "frames": a.frames, "fpl": fpl, "tuning": json.loads(g), "stripes": n,
                       "stripe_rows": a.stripe_rows, "share_ms_max": max(ms), "share_ms_mean": round(sum(ms) / len(ms), 3),
                       "max_over_mean": round(max(ms) / (sum(ms) / len(ms)), 4),
                       "job_Msamples_s": round(w * h * a.frames * depth / (max(ms) / 1e3) / 1e6, 1)}
                print(json.dumps(job), flush=True)
                out.append(job)
    if a.json:
        with open(a.json, "a") as fh:
            for r in out:
                fh.write(json.dumps(r) + "\n")
    rnd.set_tuning()
    dsc.close()
    rnd.close()


if __name__ == "__main__":
    main()
