"""Per-phase latency of k_render (diagnostics): with the MCPT_PHASE_TIMING
library (MCPT_LIB_OVERRIDE=.../libmcpt_hip_timing.so) and stats on, prints the
shader-clock ticks one wave spends per execution of each phase (fetch, T, L,
S), the phase executions per wave iteration and the implied clock, for a
workload and one rank's share of an N-stripe job.

    MCPT_LIB_OVERRIDE=$PWD/montecarlopathtracing_amd/lib/libmcpt_hip_timing.so \
        python tools/phase_probe.py --workload C2 --frames 20 --stripes 1,8
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import bench  # noqa: E402
from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C2", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--stripes", default="1,8")
    ap.add_argument("--tuning", default="")
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    data, camj = bench.load_scene(a.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(0)
    dsc, _ = bench.upload_scene(rnd, data)
    dsc.schedule = L.SCHED_PAIRED
    if a.tuning:
        rnd.set_tuning(**{k: int(v) for k, v in (x.split("=") for x in a.tuning.split(","))})
    st = rnd.new_state(wl["w"], wl["h"])
    for n in (int(x) for x in a.stripes.split(",")):
        rnd.set_stats(False)
        rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, a.frames, stripe_count=n)
        ms = rnd.stats()["kernel_ms"]
        rnd.set_stats(True)
        rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, a.frames, stripe_count=n)
        c = rnd.stats()
        rnd.set_stats(False)
        ph = c["phase_ticks"]
        wit = max(c["wave_iterations"], 1)
        execs = [wit, c["wave_node_phases"], c["wave_leaf_phases"], c["wave_shade_phases"]]
        seg = max(c["segments"], 1)
        rec = {"workload": a.workload, "stripes": n, "kernel_ms": round(ms, 3), "kernel_ms_stats": round(c["kernel_ms"], 3),
               "segments": seg, "wave_iterations": wit,
               "ticks_per_iteration": round(sum(ph) / wit, 1),
               "ticks_per_exec_fetch_T_L_S": [round(p / max(e, 1), 1) for p, e in zip(ph, execs)],
               "execs_per_iteration_T_L_S": [round(e / wit, 3) for e in execs[1:]],
               "iters_per_seg": round(wit * 64.0 / seg, 3),
               "lane_idle_frac": round(c["lane_idle"] / (64.0 * wit), 4),
               "frames_per_block": c["frames_per_block"]}
        print(json.dumps(rec), flush=True)
    dsc.close()
    rnd.close()


if __name__ == "__main__":
    main()
