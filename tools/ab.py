"""Interleaved A/B timing of two builds of libmcpt_hip.so (speed only).

    python tools/ab.py --libs montecarlopathtracing_amd/lib/libmcpt_hip_prev.so,montecarlopathtracing_amd/lib/libmcpt_hip.so \
        --workload C2 --frames 64 --rounds 3 --reps 3

Each round starts one child process per library (in turn, MCPT_LIB_OVERRIDE)
that renders `reps` calls of `frames` frames with the default launch plan and
prints the kernel ms of each; the median per library over all rounds is
reported.  Only the render entry points common to every build are used.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, ROOT)
    import torch  # noqa: F401
    import bench
    from montecarlopathtracing_amd import _lib as L
    from montecarlopathtracing_amd import render as R
    from montecarlopathtracing_amd import scene as S
    wl = bench.WORKLOADS[a.workload]
    data, camj = bench.load_scene(a.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(0)
    dsc, _ = bench.upload_scene(rnd, data)
    dsc.schedule = L.SCHED_PAIRED if a.schedule == "paired" else L.SCHED_SINGLE
    if a.tuning:
        rnd.set_tuning(**{k: int(v) for k, v in (x.split("=") for x in a.tuning.split(","))})
    st = rnd.new_state(wl["w"], wl["h"])
    rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, 4, frames_per_launch=a.fpl, stripe_count=a.stripes, stripe_index=a.stripe_index)
    ms = []
    for _ in range(a.reps):
        rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, a.frames, frames_per_launch=a.fpl,
                          stripe_count=a.stripes, stripe_index=a.stripe_index)
        ms.append(rnd.stats()["kernel_ms"])
    print("AB_RESULT " + json.dumps(ms), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--workload", default="C2")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--fpl", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--schedule", default="paired", choices=["single", "paired"])
    ap.add_argument("--tuning", default="", help="set_tuning knobs for every library, e.g. shade_threshold=40,fetch_threshold=8")
    ap.add_argument("--stripes", type=int, default=1, help="rank 0's share of an N-rank strong-scaled job")
    ap.add_argument("--stripe-index", type=int, default=0, help="with --stripes: this rank's share")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    libs = a.libs.split(",")
    res = {l: [] for l in libs}
    for _ in range(a.rounds):
        for lib in libs:
            env = dict(os.environ, MCPT_LIB_OVERRIDE=os.path.abspath(lib))
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--libs", lib,
                                  "--workload", a.workload, "--frames", str(a.frames), "--fpl", str(a.fpl),
                                  "--schedule", a.schedule, "--tuning", a.tuning,
                                  "--reps", str(a.reps), "--stripes", str(a.stripes), "--stripe-index", str(a.stripe_index)],
                                 env=env, capture_output=True, text=True, timeout=600)
            line = [x for x in out.stdout.splitlines() if x.startswith("AB_RESULT ")]
            if out.returncode != 0 or not line:
                print(out.stdout[-2000:], out.stderr[-2000:])
                sys.exit(1)
            res[lib] += json.loads(line[0][len("AB_RESULT "):])
            print("progress", os.path.basename(lib), line[0][len("AB_RESULT "):], flush=True)
    wl = __import__("bench").WORKLOADS[a.workload] if ROOT in sys.path else None
    for lib in libs:
        ts = sorted(res[lib])
        print(json.dumps({"lib": os.path.basename(lib), "workload": a.workload, "frames": a.frames, "fpl": a.fpl,
                          "stripes": a.stripes, "stripe_index": a.stripe_index,
                          "schedule": a.schedule,
                          "kernel_ms_median": round(ts[len(ts) // 2], 3), "kernel_ms_min": round(ts[0], 3),
                          "n": len(ts)}), flush=True)


if __name__ == "__main__":
    main()
