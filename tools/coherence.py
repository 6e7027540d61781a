"""Secondary-ray coherence experiment (round-3 review, next step 1a).

Question: does a gather's cost on C2 fall enough when the rays a wave traces
are similar (sorted by origin and direction) to pay for regrouping rays
between bounces?  The render's own rays are used: C2's cbox (diffuse-only,
the GPU-treelet tree), 1024x1024 primary rays run through the wavefront
kernels (mcpt_generate_rays, mcpt_intersect, mcpt_shade) bounce by bounce;
after bounce b the live rays (not terminated) are compacted and
mcpt_intersect (k_intersect, EXACT: one ray per lane, the same
traverse_exact k_render runs) is timed on them in several orders:

  pixel     compacted in pixel order (what a wave of 8x8 tiles holds at a
            pixel's first bounce)
  shuffle   a random permutation (what k_render's lanes hold after their
            paths desynchronise)
  morton    origin Morton code (30 bits over the scene box)
  oct       direction octant, then origin Morton
  dir       direction cube-map cell (6 faces x 16 x 16), then origin Morton
  morton_dir origin Morton (5 bits per axis), then direction cell (6 x 8 x 8)

Every order gives the same hits (checked byte for byte after undoing the
permutation).  Device time per call from HIP events on the launch stream,
median of --reps.  Run under rocprofv3 --pmc for TD/TA busy and L1 accesses
per dispatch (the dispatches are in the order printed).

    python tools/coherence.py [--bounces 1,3] [--reps 7] [--out gpurun_out/coherence.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def morton3(q):
    """Interleave three 10-bit integer columns (n, 3) -> uint32 codes."""
    def part(v):
        v = v.astype(np.uint32) & np.uint32(0x3FF)
        v = (v | (v << np.uint32(16))) & np.uint32(0x030000FF)
        v = (v | (v << np.uint32(8))) & np.uint32(0x0300F00F)
        v = (v | (v << np.uint32(4))) & np.uint32(0x030C30C3)
        v = (v | (v << np.uint32(2))) & np.uint32(0x09249249)
        return v
    return (part(q[:, 0]) << np.uint32(2)) | (part(q[:, 1]) << np.uint32(1)) | part(q[:, 2])


def dir_cell(d, k):
    """Cube-map cell of unit directions: face (0-5) * k * k + u * k + v."""
    a = np.abs(d)
    ax = np.argmax(a, axis=1)
    neg = d[np.arange(len(d)), ax] < 0
    face = ax * 2 + neg
    m = a[np.arange(len(d)), ax]
    uv = np.stack([d[np.arange(len(d)), (ax + 1) % 3], d[np.arange(len(d)), (ax + 2) % 3]], 1) / m[:, None]
    cell = np.clip(((uv + 1.0) * 0.5 * k).astype(np.int64), 0, k - 1)
    return (face * k * k + cell[:, 0] * k + cell[:, 1]).astype(np.int64)


def orders(o, d, lo, hi, rng):
    n = len(o)
    q = np.clip((o - lo) / np.maximum(hi - lo, 1e-30) * 1024.0, 0, 1023).astype(np.int64)
    mort = morton3(q).astype(np.int64)
    oct_ = ((d[:, 0] < 0).astype(np.int64) << 2) | ((d[:, 1] < 0).astype(np.int64) << 1) | (d[:, 2] < 0)
    q5 = q >> 5
    mort5 = morton3(q5).astype(np.int64)
    out = {
        "pixel": np.arange(n),
        "shuffle": rng.permutation(n),
        "morton": np.argsort(mort, kind="stable"),
        "oct": np.argsort((oct_ << 30) | mort, kind="stable"),
        "dir": np.argsort((dir_cell(d, 16) << 30) | mort, kind="stable"),
        "morton_dir": np.argsort((mort5 << 12) | dir_cell(d, 8), kind="stable"),
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bounces", default="1,3")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "coherence.json"))
    a = ap.parse_args()
    import bench
    from montecarlopathtracing_amd import _lib as L
    from montecarlopathtracing_amd import render as R
    from montecarlopathtracing_amd import scene as S
    data, camj = bench.load_scene("C2")
    cam = S.parse_camera(camj)
    rnd = R.Renderer(0)
    dsc = rnd.upload(data)
    w = h = 1024
    n = w * h
    lo = data.nodes[0]["bbmin"][:3].astype(np.float64)
    hi = data.nodes[0]["bbmax"][:3].astype(np.float64)
    rays = rnd.generate_rays(cam, w, h)
    color = torch.ones((n, 4), dtype=torch.float32, device=rnd.device)
    seeds = torch.from_numpy(R.default_seeds(n).view(np.int32)).to(rnd.device)
    want = sorted(int(x) for x in a.bounces.split(","))
    rng = np.random.default_rng(7)
    results = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for b in range(1, max(want) + 1):
        hits = rnd.intersect(dsc, rays)
        rnd.shade(dsc, rays, hits, color, seeds, 8)
        if b not in want:
            continue
        rec = R.records(rays, L.RAY)
        alive = (rec["origin"][:, 3].view(np.int32) & np.int32(L.TERMINATED - (1 << 32))) == 0
        live = np.ascontiguousarray(rec[alive])
        o = live["origin"][:, :3].astype(np.float64)
        d = live["direction"][:, :3].astype(np.float64)
        ref_hits = None
        for name, perm in orders(o, d, lo, hi, rng).items():
            rd = R.to_device(np.ascontiguousarray(live[perm]), rnd.device)
            hb = torch.zeros(len(live) * L.HIT.itemsize, dtype=torch.uint8, device=rnd.device)
            rnd.intersect(dsc, rd, hits=hb)  # warm
            ms = []
            for _ in range(a.reps):
                ev0.record()
                rnd.intersect(dsc, rd, hits=hb)
                ev1.record()
                torch.cuda.synchronize()
                ms.append(ev0.elapsed_time(ev1))
            hh = R.records(hb, L.HIT)
            back = np.empty_like(hh)
            back[perm] = hh
            if ref_hits is None:
                ref_hits = back
            same = bool(np.array_equal(back.view(np.uint8), ref_hits.view(np.uint8)))
            med = float(np.median(ms))
            r = {"bounce": b, "order": name, "rays": int(len(live)), "ms_median": round(med, 4),
                 "ms_min": round(float(min(ms)), 4), "Mrays_per_s": round(len(live) / med / 1e3, 1),
                 "hits_equal_pixel_order": same}
            results.append(r)
            print(json.dumps(r), flush=True)
    base = {(r["bounce"]): r["ms_median"] for r in results if r["order"] == "shuffle"}
    for r in results:
        r["speedup_vs_shuffle"] = round(base[r["bounce"]] / r["ms_median"], 3)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(results, fh, indent=1)
    if not all(r["hits_equal_pixel_order"] for r in results):
        print("HIT MISMATCH between orders", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
