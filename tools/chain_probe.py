"""Per-pixel chain lengths (diagnostics): every pixel's
frames are one sequential chain (one seed chain, one running mean), so an
N-rank share of a strong-scaled image cannot finish before its longest pixel
chain.  With stats on, mcpt_set_pixel_segments collects each pixel's segments
(traced or served from the primary-hit cache) over a call of F frames; this
prints their distribution and what it implies for strong scaling: the
ratio of the mean per-lane load of an N-rank share (the share's segments
over the GPU's resident lanes) to the longest chain in it.

    python tools/chain_probe.py --workload C4 --frames 64 --ranks 1,2,4,8
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import dist as D  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C4", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "chain_probe.jsonl"))
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    w, h = wl["w"], wl["h"]
    data, camj = bench.load_scene(a.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(0)
    dsc, _ = bench.upload_scene(rnd, data)
    dsc.schedule = L.SCHED_PAIRED
    st = rnd.new_state(w, h)
    counts = torch.zeros(w * h, dtype=torch.int32, device=rnd.device)
    iters = torch.zeros(w * h, dtype=torch.int32, device=rnd.device)
    rnd.set_stats(True)
    rnd.set_pixel_segments(counts, iters)
    rnd.render_frames(dsc, cam, st, wl["depth"], 1 << 30, a.frames)
    s = rnd.stats()
    rnd.set_pixel_segments(None)
    rnd.set_stats(False)
    c = counts.cpu().numpy().astype(np.int64)
    it = iters.cpu().numpy().astype(np.int64)
    pc = rnd.primary_cost()
    lanes = s["workgroups"] * 64
    assert int(c.sum()) == int(s["segments"]), (int(c.sum()), s["segments"])
    rec = {"workload": a.workload, "frames": a.frames, "pixels": w * h, "segments": int(c.sum()),
           "resident_lanes": lanes,
           "per_pixel_mean_p50_p90_p99_max": [round(float(c.mean()), 1)] + [int(np.percentile(c, q)) for q in (50, 90, 99)] + [int(c.max())],
           "max_over_mean": round(float(c.max() / c.mean()), 3)}
    shares = []
    for n in (int(x) for x in a.ranks.split(",")):
        m = D.ownership_mask(w, h, bench.STRIPE_ROWS, 0, n)
        cs = c[m]
        load = cs.sum() / float(lanes)  # segments per resident lane if perfectly balanced
        shares.append({"ranks": n, "pixels_per_lane": round(m.sum() / float(lanes), 3),
                       "mean_lane_load_segments": round(float(load), 1), "longest_chain_segments": int(cs.max()),
                       "bound": "chain" if cs.max() > load else "load",
                       "share_time_floor_vs_1gpu": round(float(max(load, cs.max()) / (c.sum() / float(lanes))), 4)})
    rec["shares"] = shares
    # how well the primary ray's own traversal cost predicts the chain's loop
    # iterations (the time a pixel's frames take at a given load)
    rec["iters_per_pixel_mean_p50_p99_max"] = [round(float(it.mean()), 1)] + [int(np.percentile(it, q)) for q in (50, 99)] + [int(it.max())]
    if pc is not None:
        pc = pc.astype(np.int64)
        rec["primary_cost_mean_p50_p99_max"] = [round(float(pc.mean()), 2)] + [int(np.percentile(pc, q)) for q in (50, 99)] + [int(pc.max())]
        rec["corr_primary_cost_vs_chain_iters"] = round(float(np.corrcoef(pc, it)[0, 1]), 4)
        top = np.argsort(it)[-1000:]  # the 1000 slowest chains
        for frac in (0.01, 0.05, 0.1):
            k = int(frac * len(pc))
            hot = np.argsort(pc, kind="stable")[-k:]
            rec["slowest1000_in_top%d%%_primary_cost" % int(frac * 100)] = int(np.isin(top, hot).sum())
        np.save(os.path.join(os.path.dirname(a.out), "chain_%s.npy" % a.workload),
                np.stack([c, it, pc]).astype(np.int32))
    print(json.dumps(rec), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "a") as fh:
        fh.write(json.dumps(rec) + "\n")
    dsc.close()
    rnd.close()


if __name__ == "__main__":
    main()
