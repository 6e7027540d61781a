"""Where a short call's fixed cost goes (diagnostics): the
timeline of every workgroup of one k_render launch, from the MCPT_PHASE_TIMING
library's wave log (mcpt_get_wave_log: start, first dry queue, end; 100 MHz
chip-wide ticks), for the bench's call shape.

    MCPT_LIB_OVERRIDE=$PWD/montecarlopathtracing_amd/lib/libmcpt_hip_timing.so \\
        python tools/tail_probe.py --workload C2 --frames 20 --fpl 0,5,10

Per launch: span (first start to last end), the start spread, when the queues
ran dry (first lane that found every queue empty) and how long workgroups
kept running after it (the tail: percentiles of end - first dry), and the
mean fraction of workgroups still running over that tail.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402


def summarize(log, ms):
    st, dry, end, last = log[:, 0], log[:, 1], log[:, 2], log[:, 3]
    t0 = st.min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731 - 100 MHz ticks -> us
    first_dry = dry.min()
    tail = (end - first_dry) / 100.0
    span = us(end.max())
    # workgroups alive over the tail, sampled on 64 points
    ts = np.linspace(first_dry, end.max(), 64)
    alive = [(end > t).mean() for t in ts]
    slow = np.argsort(end)[-16:]  # the 16 last workgroups
    ts_all = np.linspace(t0, end.max(), 128)
    alive_all = [((st <= t) & (end > t)).mean() for t in ts_all]
    return {"kernel_ms": round(ms, 3), "span_us": round(float(span), 1),
            "start_spread_us": round(float(us(st.max())), 1),
            "first_dry_us": round(float(us(first_dry)), 1),
            "tail_us_p50_p90_max": [round(float(np.percentile(tail, q)), 1) for q in (50, 90, 100)],
            "tail_share_of_span": round(float((end.max() - first_dry) / 100.0 / span), 4),
            "alive_mean_over_tail": round(float(np.mean(alive)), 4),
            "alive_mean_over_span": round(float(np.mean(alive_all)), 4),
            "last_start_after_dry_us_p50_max": [round(float(np.percentile((last - first_dry) / 100.0, 50)), 1),
                                                round(float(((last - first_dry) / 100.0).max()), 1)],
            "slowest16_last_start_after_dry_us": [round(float(x), 1) for x in (last[slow] - first_dry) / 100.0],
            "slowest16_end_after_dry_us": [round(float(x), 1) for x in (end[slow] - first_dry) / 100.0],
            "slowest16_xcd": [int(x) for x in log[slow, 7]],
            "iterations_p50_max": [int(np.percentile(log[:, 4], 50)), int(log[:, 4].max())],
            "entries_per_wg_mean": round(float(log[:, 5].mean()), 2),
            "wait_lane_iterations_mean_max": [round(float(log[:, 6].mean()), 1), int(log[:, 6].max())],
            "xcd_end_after_dry_us_max": [round(float(((end[log[:, 7] == x] - first_dry) / 100.0).max()), 1)
                                         if (log[:, 7] == x).any() else None for x in range(8)]}


def entry_summary(el, log):
    """Per-block timing of the (pixel, block) entries (the timing build's
    entry log: claim, start, end, low 32 bits of the 100 MHz clock), relative
    to the first queue-dry moment of the wave log: how long entries waited
    for their pixel's previous block, how long they ran, and the chains of
    the pixels that ended last."""
    el = el[(el[:, :, 2] != 0).all(axis=1)]  # pixels this call rendered (a share leaves the others at 0)
    dry32 = np.uint32(int(log[:, 1].min()) & 0xFFFFFFFF)
    rel = ((el.astype(np.int64) - int(dry32) + (1 << 31)) % (1 << 32) - (1 << 31)) / 100.0  # us from first dry
    claim, start, end = rel[..., 0], rel[..., 1], rel[..., 2]
    nb = el.shape[1]
    out = {"blocks": nb, "per_block": []}
    for b in range(nb):
        w = start[:, b] - claim[:, b]
        d = end[:, b] - start[:, b]
        out["per_block"].append({"block": b, "claim_us_p0_p50_p100": [round(float(np.percentile(claim[:, b], q)), 1) for q in (0, 50, 100)],
                                 "wait_us_p50_p99_max": [round(float(np.percentile(w, q)), 1) for q in (50, 99, 100)],
                                 "run_us_p50_p99_max": [round(float(np.percentile(d, q)), 1) for q in (50, 99, 100)],
                                 "end_us_p50_p99_max": [round(float(np.percentile(end[:, b], q)), 1) for q in (50, 99, 100)]})
    last_end = end.max(axis=1)
    slow = np.argsort(last_end)[-8:]
    out["slowest_pixels"] = [{"pixel": int(p), "claim": [round(float(x), 1) for x in claim[p]],
                              "start": [round(float(x), 1) for x in start[p]],
                              "end": [round(float(x), 1) for x in end[p]]} for p in slow]
    out["pixels_ending_after_dry_us_500_800_1200"] = [int((last_end > t).sum()) for t in (500, 800, 1200)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C2", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--fpl", default="0")
    ap.add_argument("--tuning", default="shade_threshold=32,fetch_threshold=8,block_entries=16")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tail_probe.jsonl"))
    ap.add_argument("--stripes", type=int, default=1, help="render one rank's share: 16-row stripes dealt to this many ranks")
    ap.add_argument("--stripe-index", type=int, default=0)
    a = ap.parse_args()
    kw = dict(stripe_count=a.stripes, stripe_index=a.stripe_index)
    wl = bench.WORKLOADS[a.workload]
    data, camj = bench.load_scene(a.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(0)
    dsc, _ = bench.upload_scene(rnd, data)
    dsc.schedule = L.SCHED_PAIRED
    if a.tuning:
        rnd.set_tuning(**{k: int(v) for k, v in (x.split("=") for x in a.tuning.split(","))})
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "a") as fh:
        for fpl in (int(x) for x in a.fpl.split(",")):
            st = rnd.new_state(wl["w"], wl["h"])
            rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, 4, frames_per_launch=fpl, **kw)  # warm
            for rep in range(3):
                rnd.drop_caches()
                rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, a.frames, frames_per_launch=fpl, **kw)
                s = rnd.stats()
                log = rnd.wave_log()
                if len(log) == 0:
                    raise SystemExit("no wave log: run with the MCPT_PHASE_TIMING library (MCPT_LIB_OVERRIDE)")
                rec = dict(workload=a.workload, frames=a.frames, fpl=fpl, frames_per_block=s["frames_per_block"],
                           stripes=a.stripes, stripe_index=a.stripe_index,
                           rep=rep, primary_ms=round(s.get("primary_ms", 0.0), 3), **summarize(log, s["kernel_ms"]))
                print(json.dumps(rec), flush=True)
                if rep == 0:
                    np.save(os.path.join(os.path.dirname(a.out), "tail_log_%s_fpl%d.npy" % (a.workload, fpl)), log)
                    el = rnd.entry_log()
                    if el is not None:
                        rec["entries"] = entry_summary(el, log)
                        print(json.dumps(rec["entries"]), flush=True)
                fh.write(json.dumps(rec) + "\n")
    dsc.close()
    rnd.close()


if __name__ == "__main__":
    main()
