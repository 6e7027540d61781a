#!/usr/bin/env python3
"""Headline benchmark: nominal Msamples/s (pixels x frames x bounces / s) of the
fused HIP path-tracing loop on BASELINE.json configs[1] (C2): Scene/cbox,
1024x1024 per GPU, 8 bounces, diffuse-only BRDF.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N       (one process per GPU)

A step = one frame: every pixel of the rank's image tile traces one sample of
up to 8 bounces and is accumulated (OpenCL::update + ColorOut once).  Scaling
is weak: each rank owns a 1024x1024 tile of a 1024 x (1024*N) image (row
stripes interleaved across ranks); no collective runs inside the timed region.
The timed region is bracketed by barrier + synchronize and the max over ranks
is reported.  Scene data, seeds and accumulators are resident in HBM before
timing starts.

Also reported (rank 0, N=1 only for cpu_baseline):
  roofline     — SURVEY.md §8(d): algorithmic bytes per active segment
                 B_seg = 328 + 64 (E_node + E_tri), E_* measured per config by
                 the CPU oracle's t-pruned left-first traversal (cached in
                 profiles/e_counts.json); achieved = B_seg x segments per launch
                 / average launch time (HIP events on the launch stream).
  cpu_baseline — the CPU oracle (plain-C restatement of the reference
                 algorithm, OpenMP) on a bounded pixel sample of the same
                 workload, on this host's cores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

STRIPE_ROWS = 16
# BASELINE.json configs: the headline is C2; C3/C5 are extra bench lines (--workload)
WORKLOADS = {
    "C2": {"desc": "C2: cbox 1024x1024/GPU, 8 bounces, diffuse-only, 1 sample/pixel/step",
           "w": 1024, "h": 1024, "depth": 8},
    "C3": {"desc": "C3: veach_mis 1024x1024/GPU, 12 bounces, glossy+emitters, 1 sample/pixel/step",
           "w": 1024, "h": 1024, "depth": 12},
    "C4": {"desc": "C4: diningroom proxy 1920x1080 (whole image over all GPUs), 16 bounces, glossy, "
                   "1 sample/pixel/step", "w": 1920, "h": 1080, "depth": 16, "strong": True},
    "C5": {"desc": "C5: 10M random triangles, 2048x2048/GPU, 8 bounces, 1 sample/pixel/step",
           "w": 2048, "h": 2048, "depth": 8},
}
W, H_PER_GPU, DEPTH = 1024, 1024, 8
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "Msamples/s (rays traced x bounces / s) at 1024x1024"


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


CBOX_CAM = {"position": [278, 273, -800], "lookat": [278, 273, -799], "up": [0, 1, 0], "fov": 39.3077}
MIS_CAM = {"position": [0, 2, 15], "lookat": [0, -2, 2.5], "up": [0, 1, 0], "fov": 28}
DINING_CAM = {"position": [-0.5, 3, 5.5], "lookat": [-0.5, 2, 0], "up": [0, 1, 0], "fov": 60}  # config.json:75-81


def load_scene(workload):
    from montecarlopathtracing_amd import scene as S
    if workload == "C2":
        return S.SceneData.from_obj(os.path.join(ROOT, "scenes/cbox/"), "cbox.obj",
                                    material_override=S.diffuse_only), CBOX_CAM
    if workload == "C3":
        return S.SceneData.from_obj(os.path.join(ROOT, "scenes/veach_mis/"), "mis.obj"), MIS_CAM
    if workload == "C4":  # synthetic stand-in for the absent geometry (tools/make_diningroom_proxy.py),
        # over the treelet tree like the reference's diningroom entry ("bvhtype": "treeletGPU")
        from montecarlopathtracing_amd import render as R
        d = S.SceneData.from_obj(os.path.join(ROOT, "scenes/diningroom/"), "diningroom.obj")
        return d.with_nodes(R.treelet_device(d.nodes)), DINING_CAM
    if workload == "C5":
        return S.random_mesh(10_000_000), S.RANDOM_MESH_CAMERA
    raise ValueError(workload)


def e_counts(workload="C2"):
    """E_node / E_tri (per active segment) of the t-pruned, left-first
    reference traversal, measured once by the CPU oracle
    (tests/measure_e_counts.py) and committed in profiles/e_counts.json."""
    try:
        with open(os.path.join(ROOT, "profiles", "e_counts.json")) as fh:
            return json.load(fh).get(workload)
    except (OSError, ValueError):
        return None


def default_seeds(n):
    from montecarlopathtracing_amd.render import default_seeds as ds
    return ds(n)


def cpu_baseline(data, cam, h_img, target_s=15.0):
    """The CPU oracle on a bounded sample: every k-th pixel of the same image,
    same depth, frames scaled so the sample takes ~target_s seconds."""
    from tests import oracle as O
    if not O.available():
        return None
    threads = max(1, min(16, os.cpu_count() or 1))
    seeds = default_seeds(W * h_img)
    stride = 61
    px = np.arange(0, W * h_img, stride, dtype=np.int32)
    O.render(data, cam, W, h_img, DEPTH, 1, 1 << 20, seeds, pixels=px[:2048], threads=threads)  # warm
    t0 = time.time()
    O.render(data, cam, W, h_img, DEPTH, 8, 1 << 20, seeds, pixels=px, threads=threads)
    probe = max(time.time() - t0, 1e-3) / 8.0  # seconds per frame of the sample
    frames = int(max(1, min(4096, target_s / probe)))
    t0 = time.time()
    _, _, _, st = O.render(data, cam, W, h_img, DEPTH, frames, 1 << 20, seeds, pixels=px, threads=threads)
    dt = time.time() - t0
    return {"value": len(px) * frames * DEPTH / dt / 1e6, "unit": "Msamples/s", "cores": threads,
            "kind": "port",
            "sample": "every %dth pixel (%d px) of the 1024x1024 C2 image x %d frames x depth %d, %.1f s; "
                      "oracle/mcpt_oracle.c exhaustive reference traversal, %d OpenMP threads" % (
                          stride, len(px), frames, DEPTH, dt, threads),
            "active_Msegments_per_s": float(st[0]) / dt / 1e6}


def load_traffic(workload, steps):
    """Memory-side bytes per launch of the hot kernel from the committed
    rocprofv3 PMC summary (tools/summarize_profiles.py), for this workload
    and launch size only; None otherwise."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            j = json.load(fh).get(workload) or {}
    except (OSError, ValueError):
        return None
    return j.get("hbm_bytes_per_launch") if j.get("frames_per_launch") == steps else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames per pixel block; 0 = the library's load-balance choice (4..16)")
    ap.add_argument("--workload", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--schedule", default="auto", choices=["auto", "single", "paired"],
                    help="k_render leaf-test schedule; auto times both before the warmup (untimed)")
    args = ap.parse_args()
    global W, H_PER_GPU, DEPTH
    wl = WORKLOADS[args.workload]
    W, H_PER_GPU, DEPTH = wl["w"], wl["h"], wl["depth"]

    ws, rank, local = dist_env()
    n = max(ws, 1)
    # MCPT_BENCH_SHARED_GPU=1 rehearses the N-rank path on a one-GPU box: every
    # rank on device 0, gloo for the barrier / max-reduce (tests/test_gpu_bench.py)
    shared = os.environ.get("MCPT_BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from montecarlopathtracing_amd import _lib as L
    from montecarlopathtracing_amd import render as R
    from montecarlopathtracing_amd import scene as S

    strong = bool(wl.get("strong"))
    h_img = H_PER_GPU if strong else H_PER_GPU * n  # strong: one fixed image striped over the ranks
    data, camj = load_scene(args.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(local if ws > 1 else 0)
    dsc = rnd.upload(data)
    seeds = default_seeds(W * h_img)
    st = rnd.new_state(W, h_img, seeds)
    kw = dict(stripe_rows=STRIPE_ROWS, stripe_index=rank, stripe_count=n, frames_per_launch=args.frames_per_launch)
    attempt = 1 << 30  # accumulate every frame (the reference's MAX_ATTEMPT cap never binds here)
    # leaf-test schedule (identical images; speed only), chosen before any timing
    if args.schedule == "auto":
        # timed on calls of the timed call's size (same frame-block regime), 3 trials each
        rnd.tune_schedule(dsc, cam, st, DEPTH, attempt, frames=max(1, min(args.steps, 64)), trials=3, **kw)
    else:
        dsc.schedule = L.SCHED_PAIRED if args.schedule == "paired" else L.SCHED_SINGLE

    # warmup (untimed)
    if args.warmup > 0:
        rnd.render_frames(dsc, cam, st, DEPTH, attempt, args.warmup, **kw)
    # snapshot for the segment-count replay
    snap = (st.seeds.clone(), st.hist.clone(), st.count.clone(), st.frames_done)
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rnd.render_frames(dsc, cam, st, DEPTH, attempt, args.steps, **kw)
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    kst = rnd.stats()
    kernel_ms, launches = kst["kernel_ms"], max(kst["launches"], 1)
    fpb = kst["frames_per_block"]
    if ws > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else rnd.device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    # replay the same frames with counters on (deterministic: same segments)
    st.seeds.copy_(snap[0]), st.hist.copy_(snap[1]), st.count.copy_(snap[2])
    st.frames_done = snap[3]
    rnd.set_stats(True)
    rnd.render_frames(dsc, cam, st, DEPTH, attempt, args.steps, **kw)
    cst = rnd.stats()
    rnd.set_stats(False)
    segments = cst["segments"]

    # the job's one exchange, after the timed frames: every rank's row stripes
    # summed onto rank 0 (dist.reduce_image: RCCL over xGMI; gloo when rehearsed
    # on a shared GPU), timed on its own and reported beside the frame rate
    reduce_ms = None
    if ws > 1:
        from montecarlopathtracing_amd import dist as D
        mask = D.ownership_mask(W, h_img, STRIPE_ROWS, rank, n)
        bufs = (st.hist, st.count, st.seeds)
        if shared:  # gloo: host copies
            bufs = tuple(b.cpu() for b in bufs)
        torch.cuda.synchronize()
        torch.distributed.barrier()
        t1 = time.perf_counter()
        D.reduce_image(*bufs, mask)
        torch.cuda.synchronize()
        torch.distributed.barrier()
        reduce_ms = (time.perf_counter() - t1) * 1e3

    total_samples = float(W * h_img) * args.steps * DEPTH
    value = total_samples / elapsed / 1e6
    out = None
    if rank == 0:
        ec = e_counts(args.workload)
        roof = None
        if ec:
            b_seg = 328.0 + 64.0 * (ec["E_node"] + ec["E_tri"])
            seg_per_launch = segments / float(launches)
            avg_launch_s = kernel_ms / 1e3 / launches
            achieved = b_seg * seg_per_launch / avg_launch_s / 1e9
            traffic = load_traffic(args.workload, args.steps)
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "B_seg": round(b_seg, 1), "E_node": round(ec["E_node"], 3), "E_tri": round(ec["E_tri"], 3),
                    "segments_per_launch": int(seg_per_launch), "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                    "kernel": "k_render<EXACT, no stats, %s>" % ("paired" if dsc.schedule == L.SCHED_PAIRED else "single"),
                    "kernel_node_fetches_per_seg": round(cst["node_visits"] / max(segments, 1), 3),
                    "kernel_tri_tests_per_seg": round(cst["tri_tests"] / max(segments, 1), 3)}
            # the records this kernel itself gathers per segment (128-B 4-wide
            # nodes, 64-B triangles, 48 B of pixel state per pixel-launch):
            # frac > 1 above means the kernel needs fewer bytes than the
            # reference traversal's B_seg, not that it beats HBM
            own = (128.0 * cst["node_visits"] + 64.0 * cst["tri_tests"]
                   + 48.0 * W * h_img / n * max(cst["launches"], 1)) / max(segments, 1)
            roof["own_bytes_per_seg"] = round(own, 1)
            roof["own_achieved"] = round(own * seg_per_launch / avg_launch_s / 1e9, 1)
            roof["own_frac"] = round(roof["own_achieved"] / HBM_PEAK_GBS, 4)
            # the measured streaming-read bandwidth beside the spec
            try:
                roof["measured_read_peak"] = round(rnd.measure_read_bw(4 << 30), 1)
            except Exception as e:  # reported, never fatal to the bench line
                roof["measured_read_peak"] = "unavailable: %s" % e
        cpu = None
        if n == 1 and not args.no_cpu and args.workload == "C2":
            cpu = cpu_baseline(data, cam, h_img)
        out = {"metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": n, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
               "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
               "dtype": "f32",
               "data": "synthetic seeds; " + ("Scene/cbox geometry recovered from the reference's cbox.mb"
                                              if args.workload == "C2" else "see config.workload"),
               "config": {"workload": wl["desc"],
                          "width": W, "height_per_gpu": h_img // n if strong else H_PER_GPU, "max_depth": DEPTH,
                          "parallelism": "row-stripe tiles x%d" % n, "mode": "exact",
                          "schedule": "paired" if dsc.schedule == L.SCHED_PAIRED else "single",
                          "frames_per_block": fpb},
               "active_Msegments_per_s": round(segments * n / elapsed / 1e6, 2),
               "image_reduce_ms": None if reduce_ms is None else round(reduce_ms, 3),
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    dsc.close()
    rnd.close()
    if ws > 1:
        torch.distributed.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
