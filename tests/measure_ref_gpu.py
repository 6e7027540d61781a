"""Test infrastructure: the reference's OWN kernels (oracle/_ref: rayGenerator,
intersect, shade, history.cl compiled unmodified for gfx950, replayed as
OpenCL::update by tests/refgpu.py) timed on the GPU box, on the bench's
workloads and scenes -- the reference's speed on the same MI355X, for
DESIGN.md beside the HIP path's.

    python tests/measure_ref_gpu.py [--workloads C2,C3,C4,C5] [--json out.jsonl]

Each workload renders the bench's image at the bench's depth for f1 and f2
frames (one ref_render call each: scene upload, per-frame kernel launches,
one download); the rate is the extra frames' samples over the extra time,
so the upload and download cancel out.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import refgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="C2,C3,C4")
    ap.add_argument("--frames", default="8,40")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    f1, f2 = (int(x) for x in a.frames.split(","))
    frames_for = {"C5": (1, 3)}  # 10 M triangles, traversed exhaustively: seconds per frame
    out = []
    for wl_name in a.workloads.split(","):
        wl = bench.WORKLOADS[wl_name]
        w, h, depth = wl["w"], wl["h"], wl["depth"]
        data, camj = bench.load_scene(wl_name)  # the GPU-treelet tree the bench renders over
        if data.nodes is None:  # C5: HLBVH and GPU treelet pass built on the GPU as bench.upload_scene builds them
            dt = R.to_device(data.tris, 0)
            dn = R.build_hlbvh_device(dt)
            R.treelet_gpu_device(dn)
            data = data.with_nodes(R.records(dn, L.BVHNODE).copy())
            del dt, dn
        cam = S.parse_camera(camj)
        g1, g2 = frames_for.get(wl_name, (f1, f2))
        seeds = R.default_seeds(w * h)
        refgpu.render(data, cam, w, h, depth, 2, bench.ATTEMPT, seeds)  # warm: code objects, allocations
        ts = {}
        for f in (g1, g2, g1, g2):
            t0 = time.perf_counter()
            refgpu.render(data, cam, w, h, depth, f, bench.ATTEMPT, seeds)
            ts.setdefault(f, []).append(time.perf_counter() - t0)
        t1, t2 = min(ts[g1]), min(ts[g2])
        rate = w * h * (g2 - g1) * depth / (t2 - t1) / 1e6
        rec = {"workload": wl_name, "width": w, "height": h, "max_depth": depth, "frames": [g1, g2],
               "wall_s": [round(t1, 4), round(t2, 4)], "ms_per_frame": round((t2 - t1) * 1e3 / (g2 - g1), 3),
               "Msamples_s": round(rate, 1),
               "note": "the reference's own OpenCL kernels (unmodified, gfx950) replaying OpenCL::update: "
                       "generateRay, maxdepth x (intersectRays, shade), history per frame, on this MI355X"}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if a.json:
        with open(a.json, "a") as fh:
            for r in out:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
