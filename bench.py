#!/usr/bin/env python3
"""Headline benchmark: nominal Msamples/s (pixels x frames x bounces / s) of the
fused HIP path-tracing loop on BASELINE.json configs[1] (C2): Scene/cbox,
1024x1024 per GPU, 8 bounces, diffuse-only BRDF.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N       (one process per GPU)

A step = one frame: every pixel of the image traces one sample of up to 8
bounces and is accumulated (OpenCL::update + ColorOut once).  The path
partitions (pixels are independent; 16-row stripes dealt round-robin to the
ranks, no data-path collective), so at N > 1 the headline is weak scaling:
each rank renders a 1024x1024 share of a 1024 x 1024N image — the C2 config
per GPU — and value = all ranks' samples / the slowest rank's time.  The
strong-scaled rate (the fixed 1024x1024 image striped over the ranks) is
timed after it and reported under "strong_scaling" (C4, a fixed 1920x1080
image tile-sharded across the GPUs, is strong-scaled as its config says).
No collective runs inside the timed region.  The timed region
is bracketed by barrier + synchronize and the max over ranks is reported.
Scene data, seeds and accumulators are resident in HBM before timing starts.
The timed call computes its own primary hits (k_primary, then k_render reads
them at every frame start): nothing the warmup computed is reused.

Also reported (rank 0; cpu_baseline at N=1 only):
  roofline     — the hot kernel k_render against HBM (bound "hbm", the
                 contract's roofline): traffic = memory-side bytes per launch
                 (rocprofv3 FETCH_SIZE x the calibrated scale + WRITE_SIZE of
                 this same command's timed launch, committed in
                 profiles/pmc_summary.json by tools/profile.py), achieved =
                 traffic / the launch's device time measured here (HIP events
                 on the launch stream), frac = achieved / 8 TB/s.  On the
                 cache-resident scenes HBM does not bind: the unit that does,
                 the vector-memory data path (binding_unit "td"), is reported
                 in roofline.td -- frac = TD busy cycles per CU per cycle (<= 1),
                 beside it the busy fraction of the saturating microbenchmark
                 and the floor of the TD model fitted on every committed
                 profile (profiles/td_floor_fit.json) -- with the gather fill
                 of the kernel's own counters (lanes per T-phase node gather,
                 tests per L phase), issue_frac (VALU busy x lane use) and the
                 L1/L2 hit rates.  ref_traversal_equiv_GBps restates the rate
                 in SURVEY.md §8(d)'s B_seg units (bytes the reference's
                 traversal would move per segment); it is not HBM traffic.
  cpu_baseline — the CPU oracle (plain-C restatement of the reference
                 algorithm, OpenMP on every core this process may use) on a
                 bounded pixel sample of the same workload.
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
    "C2": {"desc": "C2: cbox 1024x1024, 8 bounces, diffuse-only, 1 sample/pixel/step",
           "w": 1024, "h": 1024, "depth": 8},
    "C3": {"desc": "C3: veach_mis 1024x1024, 12 bounces, glossy+emitters, 1 sample/pixel/step",
           "w": 1024, "h": 1024, "depth": 12},
    "C4": {"desc": "C4: diningroom proxy 1920x1080, 16 bounces, glossy, 1 sample/pixel/step",
           "w": 1920, "h": 1080, "depth": 16, "strong": True},
    "C5": {"desc": "C5: 10M random triangles, 2048x2048, 8 bounces, 1 sample/pixel/step",
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
    """The workload's scene over the tree the reference renders over: SceneCL
    restructures a fresh HLBVH with its GPU treelet kernel for every bvhtype
    (scenebuild.cpp:87-95), here mcpt_treelet_gpu_device."""
    from montecarlopathtracing_amd import render as R
    from montecarlopathtracing_amd import scene as S
    if workload == "C2":
        d, cam = S.SceneData.from_obj(os.path.join(ROOT, "scenes/cbox/"), "cbox.obj",
                                      material_override=S.diffuse_only), CBOX_CAM
    elif workload == "C3":
        d, cam = S.SceneData.from_obj(os.path.join(ROOT, "scenes/veach_mis/"), "mis.obj"), MIS_CAM
    elif workload == "C4":  # synthetic stand-in for the absent geometry (tools/make_diningroom_proxy.py)
        d, cam = S.SceneData.from_obj(os.path.join(ROOT, "scenes/diningroom/"), "diningroom.obj"), DINING_CAM
    elif workload == "C5":  # the BVH is built on the GPU at upload (upload_scene)
        return S.random_mesh(10_000_000, build=lambda t: None), S.RANDOM_MESH_CAMERA
    else:
        raise ValueError(workload)
    return d.with_nodes(R.treelet_gpu_device(d.nodes)), cam


def upload_scene(rnd, data):
    """SceneBuild::buildScene.  A scene whose BVH is not built yet (C5): the
    triangles go to HBM and everything else is built there — HLBVH, the GPU
    treelet pass, the search trees (mcpt_scene_upload_device); returns the
    scene and that build's wall time."""
    from montecarlopathtracing_amd import render as R
    if data.nodes is not None:
        return rnd.upload(data), None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dt = R.to_device(data.tris, rnd.device.index or 0)
    dn = R.build_hlbvh_device(dt)
    R.treelet_gpu_device(dn)
    dsc = rnd.upload((dt, dn, data.mats))
    torch.cuda.synchronize()
    return dsc, time.perf_counter() - t0


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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs this process may keep busy: the cgroup v2 quota (cpu.max) when one
    is set, else None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        return None


def cpu_baseline(data, cam, h_img, target_s=15.0, label="C2"):
    """The CPU oracle on a bounded sample: every k-th pixel of the same image,
    same depth, frames scaled so the sample takes ~target_s seconds, on every
    core this process may run on (all host cores)."""
    from tests import oracle as O
    if not O.available():
        return None
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = cpu_quota()
    omp = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    # every core this process may run on, capped by its CPU share (the cgroup
    # quota, or OMP_NUM_THREADS where the host sets the share that way): more
    # OpenMP threads than the share only time-slice (on the 256-core GPU box
    # with a 16-CPU share, 256 threads ran 1.7x slower than 16)
    threads = max(1, min(affinity, quota or affinity, omp or affinity))
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
            "kind": "port", "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "omp_num_threads_env": omp,
            "cpu_model": cpu_model(), "threads": threads,
            "sample": "every %dth pixel (%d px) of the %dx%d %s image x %d frames x depth %d, %.1f s; "
                      "oracle/mcpt_oracle.c exhaustive reference traversal, %d OpenMP threads" % (
                          stride, len(px), W, h_img, label, frames, DEPTH, dt, threads),
            "active_Msegments_per_s": float(st[0]) / dt / 1e6}


def _ownership(w, h, rank, n):
    from montecarlopathtracing_amd import dist as D
    return D.ownership_mask(w, h, STRIPE_ROWS, rank, n)


def load_profile(workload, steps):
    """The committed rocprofv3 summary of the timed launch of THIS command
    (workload, frames per call), written by tools/profile.py; None if that
    exact launch size was never profiled."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            return json.load(fh).get("%s@%d" % (workload, steps))
    except (OSError, ValueError):
        return None


ATTEMPT = 1 << 30  # accumulate every frame (the reference's MAX_ATTEMPT cap never binds here)


def tune_plan(rnd, dsc, cam, st, steps, kw, schedule="auto", shade_threshold=0, depth=None):
    """The launch-plan pick main() makes before the warmup (untimed; every
    setting gives the same bits): with schedule "auto", Renderer.tune over the
    leaf schedule, S and fetch thresholds, block sizing, tile order and last
    block on calls of the timed call's size, 5 trials each, every trial a
    fresh view (primary-hit pass and tile sort included, as in the timed
    call).  tests/test_gpu_fullsize.py runs this same function before
    comparing the timed call with the reference kernels.  Returns the S
    threshold in force."""
    from montecarlopathtracing_amd import _lib as L
    depth = DEPTH if depth is None else depth
    frames = max(1, min(steps, 64))
    shade_th = rnd.get_tuning()["shade_threshold"] or 32
    if schedule == "auto" and shade_threshold > 0:
        rnd.tune_schedule(dsc, cam, st, depth, ATTEMPT, frames=frames, trials=5, **kw)
    elif schedule == "auto":
        _, shade_th, _ = rnd.tune(dsc, cam, st, depth, ATTEMPT, frames=frames, trials=5, fresh_view=True, **kw)
    else:
        dsc.schedule = L.SCHED_PAIRED if schedule == "paired" else L.SCHED_SINGLE
    return shade_th


def timed_render(rnd, dsc, cam, st, steps, warmup, kw, ws, shared, depth=None, per_rank=False):
    """W untimed warmup frames, then K frames timed between barrier +
    synchronize on both sides; returns the elapsed seconds, the max over
    ranks (per_rank: also every rank's own elapsed seconds)."""
    depth = DEPTH if depth is None else depth
    if warmup > 0:
        rnd.render_frames(dsc, cam, st, depth, ATTEMPT, warmup, **kw)
    torch.cuda.synchronize()
    # the timed call computes its own primary hits (k_primary runs inside the
    # timed region): nothing the warmup computed is reused
    rnd.drop_caches()
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rnd.render_frames(dsc, cam, st, depth, ATTEMPT, steps, **kw)
    torch.cuda.synchronize()
    own = time.perf_counter() - t0  # this rank's own share, before waiting for the others
    if ws > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    ranks = [own]
    if ws > 1:
        dev = "cpu" if shared else rnd.device
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
        if per_rank:
            mine = torch.tensor([own], dtype=torch.float64, device=dev)
            allt = [torch.zeros_like(mine) for _ in range(ws)]
            torch.distributed.all_gather(allt, mine)
            ranks = [float(x.item()) for x in allt]
    return (elapsed, ranks) if per_rank else elapsed


def one_gpu_time(rnd, dsc, cam, w, h, steps, warmup, ws, rank, depth=None, frames_per_launch=0):
    """The strong-scaled image rendered whole on ONE GPU inside the same job
    (rank 0; the other ranks wait at a barrier), timed like timed_render:
    the denominator of strong_scaling.speedup_vs_1gpu.  Same tuning as the
    shares' call; returns seconds on rank 0, None elsewhere."""
    if ws > 1:
        torch.distributed.barrier()
    out = None
    if rank == 0:
        st1 = rnd.new_state(w, h, default_seeds(w * h))
        out = timed_render(rnd, dsc, cam, st1, steps, warmup,
                           dict(stripe_rows=STRIPE_ROWS, stripe_index=0, stripe_count=1,
                                frames_per_launch=frames_per_launch), 1, True, depth=depth)
        del st1
    if ws > 1:
        torch.distributed.barrier()
    return out


def strong_record(w, h, steps, elapsed, ranks, one_s, note):
    """strong_scaling: the fixed image's rate over the ranks, each rank's own
    share time, and the speed-up over the same image on one GPU in this job."""
    return {"value": round(float(w * h) * steps * DEPTH / elapsed / 1e6, 2), "unit": "Msamples/s",
            "ms_per_step": round(elapsed * 1e3 / steps, 4), "image": [w, h],
            "share_ms_per_rank": [round(x * 1e3, 3) for x in ranks],
            "share_max_over_mean": round(max(ranks) / (sum(ranks) / len(ranks)), 4),
            "one_gpu_ms": None if one_s is None else round(one_s * 1e3, 3),
            "one_gpu_value": None if one_s is None else round(float(w * h) * steps * DEPTH / one_s / 1e6, 2),
            "speedup_vs_1gpu": None if one_s is None else round(one_s / elapsed, 4),
            "note": note}


def c4_strong_leg(rnd, ws, rank, n, shared, args):
    """N > 1, the C2 headline: C4's fixed 1920x1080 image (the dining proxy,
    depth 16) striped over the ranks and rendered whole by rank 0 alone in the
    same job, with the library's auto plan; its strong_record."""
    global DEPTH
    from montecarlopathtracing_amd import scene as S
    wl = WORKLOADS["C4"]
    data, camj = load_scene("C4")
    cam = S.parse_camera(camj)
    dsc, _ = upload_scene(rnd, data)
    tuned = rnd.get_tuning()
    rnd.set_tuning()
    w, h, depth = wl["w"], wl["h"], wl["depth"]
    frames = max(1, min(args.steps, 16))
    kw = dict(stripe_rows=STRIPE_ROWS, stripe_index=rank, stripe_count=n)
    st = rnd.new_state(w, h, default_seeds(w * h))
    e, e_ranks = timed_render(rnd, dsc, cam, st, frames, 1, kw, ws, shared, depth=depth, per_rank=True)
    del st
    one = one_gpu_time(rnd, dsc, cam, w, h, frames, 1, ws, rank, depth=depth)
    rnd.set_tuning(**tuned)
    dsc.close()
    saved, DEPTH = DEPTH, depth  # strong_record prices samples at the leg's depth
    try:
        return strong_record(w, h, frames, e, e_ranks, one,
                             "C4 (dining proxy 1920x1080, depth 16, %d frames, auto plan) striped over the ranks; "
                             "speedup_vs_1gpu = the same image and call rendered whole by rank 0 alone in this job / "
                             "the striped time" % frames)
    finally:
        DEPTH = saved


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames per pixel block; 0 = the library's load-balance choice")
    ap.add_argument("--workload", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--schedule", default="auto", choices=["auto", "single", "paired"],
                    help="k_render leaf-test schedule; auto times both before the warmup (untimed)")
    ap.add_argument("--no-strong", action="store_true", help="N > 1: skip the strong-scaling legs")
    ap.add_argument("--no-c4-leg", action="store_true", help="N > 1, C2: skip C4's strong-scaling leg")
    ap.add_argument("--no-cache-off", action="store_true", help="skip the primary-cache-off timing")
    ap.add_argument("--shade-threshold", type=int, default=0,
                    help="k_render S-phase threshold (mcpt_tuning.shade_threshold); 0: tuned with the schedule "
                         "when --schedule is auto, else the default")
    ap.add_argument("--fetch-threshold", type=int, default=0,
                    help="k_render fetch threshold (mcpt_tuning.fetch_threshold); 0: tuned like the S threshold")
    ap.add_argument("--block-entries", type=int, default=0,
                    help="k_render block sizing (mcpt_tuning.block_entries); 0: tuned like the S threshold")
    ap.add_argument("--last-block-frames", type=int, default=0,
                    help="k_render last block length (mcpt_tuning.last_block_frames, -1 equal blocks); "
                         "0: tuned like the S threshold")
    ap.add_argument("--tile-order", type=int, default=-1,
                    help="k_render queue tile order (mcpt_tuning.tile_order: 0 dearest first by the costliest "
                         "pixel, 1 image order, 2 by summed cost); -1: tuned with the block sizing")
    ap.add_argument("--quantized", type=int, default=0, choices=[0, 1, 2],
                    help="EXACT search-tree format (mcpt_tuning.quantized: 0 auto, 1 the 64-B quantized nodes, "
                         "2 the 128-B nodes)")
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
    # one rank per GPU: a node with fewer visible GPUs than ranks is refused
    # here, before any call that initialises a device (device_count does not)
    if ws > 1 and not shared and (torch.cuda.device_count() < ws or local >= torch.cuda.device_count()):
        print("bench.py: WORLD_SIZE %d needs %d visible GPUs (one per rank), %d visible" % (
            ws, ws, torch.cuda.device_count()), file=sys.stderr, flush=True)
        sys.exit(3)
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

    # weak scaling (the headline): a 1024 x 1024N image, each rank a 1024x1024
    # share; C4 strong-scales its fixed image
    strong_only = bool(wl.get("strong"))
    h_img = H_PER_GPU if strong_only else H_PER_GPU * n
    data, camj = load_scene(args.workload)
    cam = S.parse_camera(camj)
    rnd = R.Renderer(local if ws > 1 else 0)
    dsc, build_s = upload_scene(rnd, data)
    seeds = default_seeds(W * h_img)
    st = rnd.new_state(W, h_img, seeds)
    kw = dict(stripe_rows=STRIPE_ROWS, stripe_index=rank, stripe_count=n, frames_per_launch=args.frames_per_launch)
    attempt = ATTEMPT
    # leaf-test schedule (identical images; speed only), chosen before any timing
    if args.shade_threshold > 0:
        rnd.set_tuning(**dict(rnd.get_tuning(), shade_threshold=args.shade_threshold))
    if args.fetch_threshold > 0:
        rnd.set_tuning(**dict(rnd.get_tuning(), fetch_threshold=args.fetch_threshold))
    if args.block_entries > 0:
        rnd.set_tuning(**dict(rnd.get_tuning(), block_entries=args.block_entries))
    if args.last_block_frames != 0:
        rnd.set_tuning(**dict(rnd.get_tuning(), last_block_frames=args.last_block_frames))
    if args.tile_order >= 0:
        rnd.set_tuning(**dict(rnd.get_tuning(), tile_order=args.tile_order))
    if args.quantized:
        rnd.set_tuning(**dict(rnd.get_tuning(), quantized=args.quantized))
    shade_th = tune_plan(rnd, dsc, cam, st, args.steps, kw, schedule=args.schedule,
                         shade_threshold=args.shade_threshold)

    elapsed, rank_s = timed_render(rnd, dsc, cam, st, args.steps, args.warmup, kw, ws, shared, per_rank=True)
    kst = rnd.stats()
    # the same frames with the primary-hit cache off (every frame traces its
    # primary ray), timed after the headline: the memoization's share of it
    cache_off = None
    if not args.no_cache_off:
        base_tuning = rnd.get_tuning()
        rnd.set_tuning(**dict(base_tuning, primary_cache=2))
        st_off = rnd.new_state(W, h_img, seeds)
        e_off = timed_render(rnd, dsc, cam, st_off, args.steps, args.warmup, kw, ws, shared)
        rnd.set_tuning(**base_tuning)
        cache_off = {"value": round(float(W * h_img) * args.steps * DEPTH / e_off / 1e6, 2), "unit": "Msamples/s",
                     "ms_per_step": round(e_off * 1e3 / args.steps, 4),
                     "note": "mcpt_tuning.primary_cache = 2: every frame traces its primary ray (same bits)"}
        del st_off
    # the boundary keeps the image state in HBM across calls (the reference's
    # OpenCL buffers live on its device too); host copies happen only at a
    # dump (ColorOut): this rank's hist/count/seeds to pinned host memory,
    # timed apart from value (PCIe-inclusive rate)
    dump = None
    if rank == 0:
        host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in (st.hist, st.count, st.seeds)]
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for hbuf, t in zip(host, (st.hist, st.count, st.seeds)):
                hbuf.copy_(t, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        dump_s = sorted(ts)[1]
        nbytes = sum(t.numel() * t.element_size() for t in (st.hist, st.count, st.seeds))
        dump = {"ms": round(dump_s * 1e3, 3), "bytes": nbytes, "GBps": round(nbytes / dump_s / 1e9, 1),
                "value_with_dump_per_call": round(float(W * h_img) * args.steps * DEPTH / (elapsed + dump_s) / 1e6, 2),
                "note": "device-to-host copy of the image state (24 B/pixel) after the call, outside value"}
        del host
    # k_render alone: the call's device time less the primary-hit pass before it
    primary_ms = kst.get("primary_ms", 0.0) if kst.get("primary_cache") == 2 else 0.0
    kernel_ms, launches = kst["kernel_ms"] - primary_ms, max(kst["launches"], 1)
    fpb = kst["frames_per_block"]
    search_tree = "64-B quantized" if kst.get("quantized") else "128-B exact"

    # replay the same frames with counters on (deterministic: same segments)
    # (the counting kernel runs the replay's warmup too, so the timed launch
    # stays the last dispatch of the non-counting kernel: tools/profile.py)
    st2 = rnd.new_state(W, h_img, seeds)
    rnd.set_stats(True)
    if args.warmup > 0:
        rnd.render_frames(dsc, cam, st2, DEPTH, attempt, args.warmup, **kw)
    rnd.render_frames(dsc, cam, st2, DEPTH, attempt, args.steps, **kw)
    cst = rnd.stats()
    rnd.set_stats(False)
    segments = cst["segments"]
    # segments whose hit the primary-hit cache served (each frame's first, no
    # traversal): this rank's pixels x frames when the call read the cache
    my_px = int(np.count_nonzero(_ownership(W, h_img, rank, n)))
    served = my_px * args.steps if cst.get("primary_cache") in (1, 2) else 0
    traced = segments - served
    del st2

    # the job's one exchange, after the timed frames: every rank's row stripes
    # summed onto rank 0 (dist.reduce_image: RCCL over xGMI; gloo when rehearsed
    # on a shared GPU), timed on its own and reported beside the frame rate
    reduce_ms = None
    strong = c4 = None
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
        if not args.no_strong and not strong_only:
            # strong scaling: the fixed 1024x1024 image striped over the ranks,
            # then the same image on one GPU (rank 0) in this same job, with the
            # headline's tuning (tuned on 1024x1024 pixels per GPU: the same
            # pixel count as the whole image on one GPU)
            sts = rnd.new_state(W, H_PER_GPU, default_seeds(W * H_PER_GPU))
            es, es_ranks = timed_render(rnd, dsc, cam, sts, args.steps, args.warmup, kw, ws, shared, per_rank=True)
            del sts
            one = one_gpu_time(rnd, dsc, cam, W, H_PER_GPU, args.steps, args.warmup, ws, rank,
                               frames_per_launch=args.frames_per_launch)
            strong = strong_record(W, H_PER_GPU, args.steps, es, es_ranks, one,
                                   "the fixed 1024x1024 image striped over the ranks; speedup_vs_1gpu = the same "
                                   "image and call rendered whole by rank 0 alone in this job / the striped time")
            if args.workload == "C2" and not args.no_c4_leg:
                c4 = c4_strong_leg(rnd, ws, rank, n, shared, args)
        elif not args.no_strong and strong_only:
            # C4: the headline IS the strong-scaled image; the one-GPU time of
            # the same call in this job, with the library's auto plan (the
            # tuning was picked for a share, not the whole image)
            tuned = rnd.get_tuning()
            rnd.set_tuning()
            one = one_gpu_time(rnd, dsc, cam, W, h_img, args.steps, args.warmup, ws, rank,
                               frames_per_launch=args.frames_per_launch)
            rnd.set_tuning(**tuned)
            strong = strong_record(W, h_img, args.steps, elapsed, rank_s, one,
                                   "the headline's fixed image; speedup_vs_1gpu = the same image and call rendered "
                                   "whole by rank 0 alone in this job (auto plan) / the striped time")

    total_samples = float(W * h_img) * args.steps * DEPTH
    value = total_samples / elapsed / 1e6
    out = None
    if rank == 0:
        avg_launch_s = kernel_ms / 1e3 / launches
        seg_per_launch = segments / float(launches)
        prof = load_profile(args.workload, args.steps) if n == 1 else None
        roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "achieved": None, "frac": None, "traffic": None,
                "kernel": "k_render<EXACT, no stats, %s, %s nodes>" % (
                    "paired" if dsc.schedule == L.SCHED_PAIRED else "single", search_tree),
                "avg_launch_ms": round(avg_launch_s * 1e3, 3), "segments_per_launch": int(seg_per_launch),
                "segments_traced": int(traced), "segments_cache_served": int(served),
                "primary_pass_ms": round(primary_ms, 3),
                # per TRACED segment: the cache-served ones fetch no node or triangle
                "kernel_node_fetches_per_seg": round(cst["node_visits"] / max(traced, 1), 3),
                "kernel_tri_tests_per_seg": round(cst["tri_tests"] / max(traced, 1), 3)}
        if prof:
            traffic = prof["hbm_bytes_per_launch"]
            roof["traffic"] = traffic
            roof["achieved"] = round(traffic / avg_launch_s / 1e9, 2)
            roof["frac"] = round(roof["achieved"] / HBM_PEAK_GBS, 5)
            # issue_frac: lane-weighted VALU use = VALU-busy cycles x the share of
            # the 64 lanes those instructions ran with (rocprofv3 VALUUtilization);
            # the raw busy ratio beside it (rocprofv3's VALUBusy definition reads
            # up to ~1 % over 1 on a saturated kernel, C3: DESIGN.md §3.6)
            vb, vu = prof.get("valu_busy"), prof.get("valu_utilization_lanes")
            roof["issue_frac"] = None if vb is None or vu is None else round(vb * vu, 4)
            roof["valu_busy"] = vb
            roof["valu_lane_utilization"] = vu
            roof["td_busy"] = prof.get("td_busy")
            roof["binding"] = ("vector-memory gathers: TD (data-return) busy %s of the kernel's cycles; VALU busy %s at "
                               "%s lane use (DESIGN.md §3.6)" % (prof.get("td_busy"), vb, vu))
            for k in ("l1_hit_rate", "l2_hit_rate", "l2_hit_GBps_128B_lines", "wave_wait_any_per_wave_cycle",
                      "gather_latency_cycles_per_vmem_rd", "fetch_scale_calibrated", "timed_launch_ms_rocprof"):
                roof[k] = prof.get(k)
            roof["profile"] = prof.get("source")
            # HBM is the roofline the contract names (bound "hbm"); on the
            # cache-resident scenes the unit that binds is the vector-memory
            # data path (TD), reported beside it (roofline.td):
            #   frac       = TD busy cycles per CU per kernel cycle (rocprofv3
            #                TD_TD_BUSY of this command's timed launch; <= 1 by
            #                construction), busy_vs_microbench = that over the
            #                saturating microbenchmark's (tools/mb/td_lanes.hip)
            #   model_floor_frac = the launch's gather instructions and L2
            #                requests at the costs fitted on every committed
            #                profile (profiles/td_floor_fit.json), / its cycles
            #   fill       = lanes per T-phase node gather (the kernel's own
            #                counters of the replay: node steps / wave T phases)
            td, fit = prof.get("td_model"), prof.get("td_fit")
            hbm = {"achieved": roof["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": roof["frac"],
                   "traffic": traffic}
            roof["hbm"] = hbm
            clk = prof.get("clock_GHz")
            if td and clk and fit:
                roof["binding_unit"] = "td"
                roof["td"] = {"achieved": round(fit["td_busy_per_cycle"] * clk, 4), "peak": round(clk, 4),
                              "unit": "G TD-busy cycles/s per CU", "frac": fit["td_busy_per_cycle"],
                              "busy_vs_microbench": td.get("busy_frac"),
                              "model_floor_frac": fit["model_frac"], "model": fit["fit"],
                              "inst_term_share_fitted": fit["inst_term_share"],
                              # the free fit's b = 0 comes from collinear data (gather instructions and
                              # line accesses correlate 0.987 across the profiles): with b held at the
                              # microbenchmark's 0.74 the share collapses; the split is not identifiable
                              # from these kernels, so all three are reported
                              "inst_term_share_b_fixed": fit.get("inst_term_share_b_fixed"),
                              "model_floor_frac_b_fixed": fit.get("model_frac_b_fixed"),
                              "inst_term_share_microbench": round(
                                  td["a_cycles_per_inst"] * td["vmem_rd_insts"] /
                                  (td["a_cycles_per_inst"] * td["vmem_rd_insts"] +
                                   td["b_cycles_per_line"] * td["l1_accesses"]), 4),
                              "a_cycles_per_gather_inst_microbench": td["a_cycles_per_inst"],
                              "b_cycles_per_line_microbench": td["b_cycles_per_line"],
                              "vmem_rd_insts": fit["vmem_rd_insts"], "l1_line_accesses": fit["l1_accesses"],
                              "l2_requests": fit["l2_requests"],
                              "l1_lines_per_vmem_rd_inst": fit["l1_lines_per_vmem_rd_inst"]}
        # gather-instruction fill from the kernel's own counters (the replay):
        # lanes per T-phase node gather and triangle tests per L phase
        roof["lanes_per_node_gather_inst"] = round(cst["node_visits"] / max(cst["wave_node_phases"], 1), 2)
        roof["tests_per_leaf_phase"] = round(cst["tri_tests"] / max(cst["wave_leaf_phases"], 1), 2)
        ec = e_counts(args.workload)
        if ec:
            b_seg = 328.0 + 64.0 * (ec["E_node"] + ec["E_tri"])
            roof["ref_traversal_equiv_GBps"] = round(b_seg * seg_per_launch / avg_launch_s / 1e9, 1)
            roof["ref_traversal_B_seg"] = round(b_seg, 1)
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
               "higher_is_better": True, "scaling": "strong" if (strong_only and n > 1) else "weak",
               "vs_baseline": None,
               "dtype": "f32",
               "data": "synthetic seeds; " + ("Scene/cbox geometry recovered from the reference's cbox.mb"
                                              if args.workload == "C2" else "see config.workload"),
               "config": {"workload": wl["desc"],
                          "width": W, "height": h_img, "max_depth": DEPTH,
                          "parallelism": "row-stripe tiles x%d" % n, "mode": "exact",
                          "schedule": "paired" if dsc.schedule == L.SCHED_PAIRED else "single",
                          "shade_threshold": shade_th,
                          "fetch_threshold": rnd.get_tuning()["fetch_threshold"] or 1,
                          "block_entries": rnd.get_tuning()["block_entries"] or 8,
                          "frames_per_block": fpb,
                          "last_block_frames": rnd.get_tuning()["last_block_frames"],
                          "tile_order": {0: "dearest first (costliest pixel)", 1: "image", 2: "dearest first (summed)"}[
                              rnd.get_tuning()["tile_order"]],
                          "search_tree_nodes": search_tree,
                          "search_tree_top_levels_in_lds": kst.get("top_levels"),
                          "stack": "16-entry LDS window + HBM spill" if kst.get("stack_window") else "whole in LDS",
                          "resident_waves": kst.get("workgroups")},
               "active_Msegments_per_s": round(segments * n / elapsed / 1e6, 2),
               "scene_build_gpu_s": None if build_s is None else round(build_s, 3),
               "traced_Msegments_per_s": round(traced * n / elapsed / 1e6, 2),
               "primary_cache_off": cache_off,
               "image_reduce_ms": None if reduce_ms is None else round(reduce_ms, 3),
               "host_dump": dump,
               "strong_scaling": strong,
               # N > 1: the strong-scaling answers at the top level, where the
               # scaling record's reader sees them (north_star: tile-parallel
               # speed-up at 1/2/4/8 GPUs): the fixed 1024x1024 image, and C4's
               # 1920x1080 image (the config north_star shards over 8 GPUs)
               "strong_speedup_vs_1gpu": None if strong is None else strong["speedup_vs_1gpu"],
               "c4_strong_speedup_vs_1gpu": (strong["speedup_vs_1gpu"] if (strong_only and strong) else
                                             (None if c4 is None else c4["speedup_vs_1gpu"])),
               "c4_strong_scaling": c4,
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    dsc.close()
    rnd.close()
    if ws > 1:
        torch.distributed.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
