"""Device-side driver over libmcpt_hip.so: the reference's OpenCL::init/update
frame loop (MCPT/OpenCLApp.cpp:36-82), RayGeneration (raygeneration.cpp),
SceneBuild/SceneCL (scenebuild.cpp) and ColorOut (colorout.cpp) on one GPU.

PyTorch only provides device memory and the stream; every kernel is the HIP
code in csrc/mcpt_device.hip.  Buffers are raw byte tensors holding the
reference's record layouts.
"""
import ctypes

import numpy as np
import torch

from . import _lib as L


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev_bytes(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def default_seeds(n, variant="splitmix"):
    """Per-pixel 32-bit seeds.  The reference draws them with srand(time); rand()
    (scenebuild.cpp:113-120) — non-deterministic — so parity runs take seeds as
    an input.  'splitmix': splitmix64(0x5EED ^ i) & 0xFFFFFFFF;
    'msvc15' keeps 15 bits like MSVC's rand()."""
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(0x5EED) ^ i) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    s = (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    if variant == "msvc15":
        s &= np.uint32(0x7FFF)
    return s


class DeviceScene:
    """SceneBuild::buildScene result living in HBM (child-box node layout).
    `data` is a host SceneData (mcpt_scene_upload), or a tuple (tris, nodes,
    mats) whose tris / nodes are device byte tensors (mcpt_scene_upload_device:
    everything built on the GPU, the same bytes)."""

    ARRAYS = ("near4", "near4q", "nodes4", "nodes", "tris", "triq")

    def __init__(self, renderer, data):
        self.renderer = renderer
        self.data = data
        self.handle = ctypes.c_void_p()
        self.schedule = L.SCHED_PAIRED  # k_render leaf-test schedule: paired measured faster on C2-C5 (tune_schedule)
        if isinstance(data, tuple):
            t, nd, mats = data
            m = np.ascontiguousarray(mats)
            n = t.numel() // L.TRIANGLE.itemsize
            L.check(L.lib().mcpt_scene_upload_device(renderer.ctx, L.ptr(t), n, L.ptr(nd), nd.numel() // L.BVHNODE.itemsize,
                                                     L.ptr(m), len(m), _stream(), ctypes.byref(self.handle)))
            return
        t = np.ascontiguousarray(data.tris)
        nd = np.ascontiguousarray(data.nodes)
        m = np.ascontiguousarray(data.mats)
        L.check(L.lib().mcpt_scene_upload(renderer.ctx, L.ptr(t), len(t), L.ptr(nd), len(nd), L.ptr(m), len(m),
                                          ctypes.byref(self.handle)))

    def read(self, which):
        """One device array as bytes (mcpt_scene_read; which: a name of ARRAYS
        or "meta" -> int32 {stack_depth, stack_depth4, quantized, n_internal})."""
        k = 6 if which == "meta" else self.ARRAYS.index(which)
        n = ctypes.c_int64()
        L.check(L.lib().mcpt_scene_read(self.handle, k, None, 0, ctypes.byref(n)))
        buf = np.zeros(n.value, np.uint8)
        L.check(L.lib().mcpt_scene_read(self.handle, k, L.ptr(buf), n.value, ctypes.byref(n)))
        return buf.view(np.int32) if which == "meta" else buf

    def close(self):
        if self.handle:
            L.lib().mcpt_scene_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ImageState:
    """Per-pixel state that persists across frames: seed chain (randBuffer),
    accumulated mean (frameBuffer) and sample count (sampleCount)."""

    def __init__(self, width, height, seeds, device):
        n = width * height
        self.width, self.height = width, height
        self.seeds = torch.from_numpy(np.ascontiguousarray(seeds, np.uint32).view(np.int32)).to(device)
        self.hist = torch.zeros((n, 4), dtype=torch.float32, device=device)
        self.count = torch.zeros(n, dtype=torch.int32, device=device)
        self.frames_done = 0

    def image(self):
        """(H, W, 4) float32 accumulated image, row 0 = bottom (GL convention)."""
        return self.hist.cpu().numpy().reshape(self.height, self.width, 4)

    def seeds_np(self):
        return self.seeds.cpu().numpy().view(np.uint32)


class Renderer:
    """One GPU context (OpenCLBasic::init equivalent)."""

    def __init__(self, device=0):
        if not torch.cuda.is_available():
            raise L.MCPTError("no GPU: the HIP path has no CPU fallback")
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        self.ctx = ctypes.c_void_p()
        L.check(L.lib().mcpt_ctx_create(device, ctypes.byref(self.ctx)))

    def close(self):
        if self.ctx:
            L.lib().mcpt_ctx_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, data):
        return DeviceScene(self, data)

    def set_stats(self, on):
        L.check(L.lib().mcpt_set_stats(self.ctx, int(bool(on))))
        self._stats_on = bool(on)

    def stats(self):
        s = L.Stats()
        L.check(L.lib().mcpt_get_stats(self.ctx, ctypes.byref(s)))
        out = {f: getattr(s, f) for f, _ in L.Stats._fields_ if f not in ("pad", "pad1")}
        out["phase_ticks"] = list(out["phase_ticks"])
        return out

    def set_pixel_segments(self, counts, iters=None):
        """mcpt_set_pixel_segments: with stats on, render calls add each pixel's
        segments into `counts` and its busy loop iterations into `iters` (int32
        CUDA tensors of width*height, zeroed by the caller; None: not
        collected)."""
        self._px_counts = (counts, iters)  # kept alive while the library holds the pointers
        n = min([t.numel() for t in (counts, iters) if t is not None], default=0)
        L.check(L.lib().mcpt_set_pixel_segments(self.ctx, None if counts is None else L.ptr(counts),
                                                None if iters is None else L.ptr(iters), n))

    def primary_cost(self):
        """mcpt_get_primary_cost: the cached view's per-pixel primary-ray
        traversal cost (uint32, width*height), or None without a cache."""
        n = ctypes.c_int64()
        L.check(L.lib().mcpt_get_primary_cost(self.ctx, None, 0, ctypes.byref(n)))
        if n.value == 0:
            return None
        out = np.zeros(n.value, np.uint32)
        L.check(L.lib().mcpt_get_primary_cost(self.ctx, L.ptr(out), n.value, ctypes.byref(n)))
        return out

    def wave_log(self):
        """mcpt_get_wave_log (MCPT_PHASE_TIMING library only): per workgroup of
        the last launch an int64 row (start, first dry, end, last entry start
        [100 MHz ticks], iterations, entries started, lane-iterations waiting,
        XCD); an empty (0, 8) array on release builds."""
        n = ctypes.c_int64()
        L.check(L.lib().mcpt_get_wave_log(self.ctx, None, 0, ctypes.byref(n)))
        if n.value == 0:
            return np.zeros((0, 8), np.int64)
        buf = np.zeros((n.value, 8), np.uint64)
        L.check(L.lib().mcpt_get_wave_log(self.ctx, L.ptr(buf), n.value, ctypes.byref(n)))
        return buf[:, [0, 1, 2, 5, 3, 4, 6, 7]].astype(np.int64)

    def entry_log(self):
        """mcpt_get_entry_log (MCPT_PHASE_TIMING library only): (pixels, blocks, 3)
        uint32 claim / start / end times (100 MHz ticks, low 32 bits) of the
        last one-launch call's queue entries; None when nothing was logged."""
        n, b = ctypes.c_int64(), ctypes.c_int32()
        L.check(L.lib().mcpt_get_entry_log(self.ctx, None, 0, ctypes.byref(n), ctypes.byref(b)))
        if n.value == 0:
            return None
        buf = np.zeros((n.value, 3), np.uint32)
        L.check(L.lib().mcpt_get_entry_log(self.ctx, L.ptr(buf), n.value, ctypes.byref(n), ctypes.byref(b)))
        return buf.reshape(-1, b.value, 3)

    def set_tuning(self, **knobs):
        """mcpt_set_tuning: k_render launch-plan knobs (leaf_threshold,
        shade_threshold, queue_chunk, block_entries, max_block_frames,
        stack_window 0 auto / 1 window / 2 whole stack, lds_pad, queues, quantized 0 auto / 1
        the 64-B search-tree nodes / 2 the 128-B ones); speed only,
        unnamed knobs take their defaults."""
        t = L.Tuning()
        for k, v in knobs.items():
            if k not in dict(L.Tuning._fields_):
                raise L.MCPTError("unknown tuning knob %r" % k)
            setattr(t, k, int(v))
        L.check(L.lib().mcpt_set_tuning(self.ctx, ctypes.byref(t)))

    def drop_caches(self):
        """mcpt_drop_caches: forget the primary-hit cache; the next render call
        recomputes (or traces) the primary hits itself."""
        L.check(L.lib().mcpt_drop_caches(self.ctx))

    def get_tuning(self):
        t = L.Tuning()
        L.check(L.lib().mcpt_get_tuning(self.ctx, ctypes.byref(t)))
        return {f: getattr(t, f) for f, _ in L.Tuning._fields_}

    def selfcheck_trig(self):
        """(angle, range) mismatch counts of the inline randomDirection sin/cos
        against the ocml calls (mcpt_selfcheck_trig); (0, 0) on a good build."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.lib().mcpt_selfcheck_trig(self.ctx, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def selfcheck_pow(self, exponents):
        """Mismatches of the Phong lobe's pow restatement against ocml's
        pow_f32 over every float in (0, 1 + 2^-10] for each exponent
        (mcpt_selfcheck_pow); 0 on a good build."""
        ys = np.ascontiguousarray(exponents, np.float32)
        n = ctypes.c_int64()
        L.check(L.lib().mcpt_selfcheck_pow(self.ctx, L.ptr(ys), len(ys), ctypes.byref(n)))
        return n.value

    def measure_read_bw(self, nbytes=4 << 30):
        """Streaming HBM read bandwidth in GB/s (mcpt_measure_read_bw)."""
        g = ctypes.c_double()
        L.check(L.lib().mcpt_measure_read_bw(self.ctx, int(nbytes), ctypes.byref(g)))
        return g.value

    def gather_probe(self, record_bytes, table_bytes=1 << 31):
        """Device ms of mcpt_gather_probe (the FETCH_SIZE calibration kernel)."""
        g = ctypes.c_double()
        L.check(L.lib().mcpt_gather_probe(self.ctx, int(record_bytes), int(table_bytes), ctypes.byref(g)))
        return g.value

    def new_state(self, width, height, seeds=None):
        if seeds is None:
            seeds = default_seeds(width * height)
        return ImageState(width, height, seeds, self.device)

    # ---------------------------------------------------------- fused path
    def render_frames(self, scene, camera, state, max_depth, max_attempt, frames, frame_begin=None,
                      stripe_rows=16, stripe_index=0, stripe_count=1, mode=L.MODE_EXACT,
                      frames_per_launch=0, schedule=None):
        """Frames [frame_begin, frame_begin+frames) for this GPU's row stripes
        (OpenCL::update x frames + ColorOut accumulation).  `schedule`
        (L.SCHED_*; default: the scene's, see tune_schedule) only changes speed."""
        p = L.RenderParams()
        p.width, p.height = state.width, state.height
        p.max_depth, p.max_attempt = int(max_depth), int(max_attempt)
        p.frame_begin = state.frames_done if frame_begin is None else int(frame_begin)
        p.frames = int(frames)
        p.stripe_rows, p.stripe_index, p.stripe_count = int(stripe_rows), int(stripe_index), int(stripe_count)
        p.mode = int(mode)
        p.frames_per_launch = int(frames_per_launch)
        p.schedule = int(getattr(scene, "schedule", L.SCHED_PAIRED) if schedule is None else schedule)
        cam = np.ascontiguousarray(camera)
        L.check(L.lib().mcpt_render_frames(self.ctx, scene.handle, L.ptr(cam), ctypes.byref(p), L.ptr(state.seeds),
                                           L.ptr(state.hist), L.ptr(state.count), _stream()))
        state.frames_done = p.frame_begin + p.frames
        return state

    def tune_schedule(self, scene, camera, state, max_depth, max_attempt, frames=64, trials=1, **kw):
        """Pick the faster leaf-test schedule for this scene and view: render
        `frames` frames `trials` times with each schedule on a scratch copy
        of `state` (interleaved, device time of each call), keep the faster
        in scene.schedule.  Both schedules give bit-identical images, so this
        only moves speed.  Returns (schedule, {schedule: best ms})."""
        sched, _, best = self.tune(scene, camera, state, max_depth, max_attempt, frames, trials, shade_thresholds=None,
                                   fetch_thresholds=None, tile_orders=None, **kw)
        return sched, {k[0]: v for k, v in best.items()}

    def tune(self, scene, camera, state, max_depth, max_attempt, frames=64, trials=1, shade_thresholds=(32, 40, 48),
             fetch_thresholds=(1, 8), block_entries=(8, 16), last_block=True, tile_orders=(0, 1, 2), fresh_view=False,
             **kw):
        """tune_schedule over the leaf-test schedule, the S-phase threshold
        (mcpt_tuning.shade_threshold) and then the fetch threshold
        (mcpt_tuning.fetch_threshold), then the block sizing
        (mcpt_tuning.block_entries) jointly with the tile order
        (mcpt_tuning.tile_order: dearest tiles first by their costliest or
        summed primary-ray cost, or image order), then a short last block
        against equal blocks (mcpt_tuning.last_block_frames -1, ceil(frames / 8)
        or ceil(frames / 4)) jointly with the block sizing again; ties keep the
        baseline value.  Their best values
        differ by scene (round 2, 3-frame blocks: veach_mis S 40, fetch 8;
        cbox S 32-40, fetch 8; the 10 M-triangle soup S 32, fetch 1; round 4:
        cbox gains 5-10 % from the dearest-first order, veach_mis loses 5 %).
        Every combination gives the same bits.  Each setting is judged by its
        median over the trials (a single timed call is what the pick has to
        predict; the minimum favoured lucky runs).  fresh_view: every trial
        call first drops the primary-hit cache, so it pays the primary-hit
        pass and the tile sort as a call of a new view does (bench.py's timed
        call).  The winner goes to
        scene.schedule and the renderer's tuning.  Returns (schedule,
        shade_threshold, {(schedule, shade, fetch, entries, tile_order): median ms})."""
        if getattr(self, "_stats_on", False):
            raise L.MCPTError("tune: counters must be off (they change the kernel)")
        base = self.get_tuning()
        ths = list(shade_thresholds) if shade_thresholds else [base["shade_threshold"]]
        scratch = ImageState.__new__(ImageState)
        scratch.width, scratch.height, scratch.frames_done = state.width, state.height, state.frames_done
        best, samples = {}, {}

        def trial(sched, th, fe, be, to):
            self.set_tuning(**dict(base, shade_threshold=th, fetch_threshold=fe, block_entries=be, tile_order=to))
            scratch.seeds, scratch.hist, scratch.count = state.seeds.clone(), state.hist.clone(), state.count.clone()
            if fresh_view:
                self.drop_caches()
            self.render_frames(scene, camera, scratch, max_depth, max_attempt, frames,
                               frame_begin=state.frames_done, schedule=sched, **kw)
            ms = self.stats()["kernel_ms"]
            samples.setdefault((sched, th, fe, be, to), []).append(ms)
            best.clear()  # median per setting: a single timed call is what the pick predicts
            best.update({k: sorted(v)[len(v) // 2] for k, v in samples.items()})

        def pick():  # fastest median; ties to the smaller key
            return min(best, key=lambda k: (best[k], k))

        fe0 = base["fetch_threshold"] or 1  # 0 = the default, 1
        be0 = base["block_entries"] or 8    # 0 = the default, 8
        to0 = base["tile_order"]
        try:
            for _ in range(int(trials)):
                for th in ths:
                    for sched in (L.SCHED_SINGLE, L.SCHED_PAIRED):
                        trial(sched, th, fe0, be0, to0)
            sched, th, fe, be, to = pick()
            if shade_thresholds and fetch_thresholds:  # then the fetch threshold, with that pair
                for _ in range(int(trials)):
                    for f in fetch_thresholds:
                        if f != fe0:
                            trial(sched, th, f, be0, to0)
                sched, th, fe, be, to = pick()
            if shade_thresholds and (block_entries or tile_orders):  # then block sizing x tile order
                bes = list(block_entries) if block_entries else [be0]
                tos = list(tile_orders) if tile_orders else [to0]
                for _ in range(int(trials)):
                    for b in bes:
                        for o in tos:
                            if (b, o) != (be0, to0):
                                trial(sched, th, fe, b, o)
                sched, th, fe, be, to = pick()
                if (be, to) != (be0, to0):  # other blocks or orders move the best S threshold (C3: 48 -> 40)
                    for _ in range(int(trials)):
                        for t in ths:
                            if t != th:
                                trial(sched, t, fe, be, to)
                    sched, th, fe, be, to = pick()
            lb = base["last_block_frames"]
            if shade_thresholds and last_block:
                # then a short last block against equal blocks, jointly with the
                # block sizing: the best last block can belong to the sizing
                # that lost with equal blocks (C2, 20 frames: (15, 5) at 8
                # entries beats 5-frame blocks at 16, which beat (10, 10))
                lbs = {-1, (int(frames) + 7) // 8, (int(frames) + 3) // 4}
                bes = sorted(set(block_entries)) if block_entries else [be]
                lsamples = {(be, lb): list(samples[(sched, th, fe, be, to)])}
                for _ in range(int(trials)):
                    for b in bes:
                        for v in sorted(lbs | {lb}):
                            if (b, v) == (be, lb):
                                continue
                            self.set_tuning(**dict(base, shade_threshold=th, fetch_threshold=fe, block_entries=b,
                                                   tile_order=to, last_block_frames=v))
                            scratch.seeds, scratch.hist, scratch.count = (state.seeds.clone(), state.hist.clone(),
                                                                          state.count.clone())
                            if fresh_view:
                                self.drop_caches()
                            self.render_frames(scene, camera, scratch, max_depth, max_attempt, frames,
                                               frame_begin=state.frames_done, schedule=sched, **kw)
                            lsamples.setdefault((b, v), []).append(self.stats()["kernel_ms"])
                lbest = {k: sorted(v)[len(v) // 2] for k, v in lsamples.items()}
                # ties go to the baseline (the sizing picked above with the auto rule's value), then the smaller key
                be, lb = min(lbest, key=lambda k: (lbest[k], k != (be, base["last_block_frames"]), k))
        finally:
            self.set_tuning(**base)
        scene.schedule = sched
        if shade_thresholds:
            self.set_tuning(**dict(base, shade_threshold=th, fetch_threshold=fe, block_entries=be,
                                   last_block_frames=lb, tile_order=to))
        return sched, th, best

    # ------------------------------------------------ wavefront (drop-in)
    def generate_rays(self, camera, width, height):
        """rayGenerator.cl: W*H Ray records (device bytes)."""
        rays = _dev_bytes(width * height * L.RAY.itemsize, self.device)
        cam = np.ascontiguousarray(camera)
        L.check(L.lib().mcpt_generate_rays(self.ctx, L.ptr(cam), width, height, L.ptr(rays), _stream()))
        return rays

    def intersect(self, scene, rays, hits=None, tmin=0.001, mode=L.MODE_EXACT):
        """intersect.cl on a ray buffer; returns the Hit buffer."""
        n = rays.numel() // L.RAY.itemsize
        if hits is None:
            hits = torch.zeros(n * L.HIT.itemsize, dtype=torch.uint8, device=self.device)
        L.check(L.lib().mcpt_intersect(self.ctx, scene.handle, L.ptr(rays), n, L.ptr(hits), float(tmin), int(mode),
                                       _stream()))
        return hits

    def shade(self, scene, rays, hits, color, seeds, max_depth):
        """shade.cl on (rays, hits, colour, seeds) in place."""
        n = rays.numel() // L.RAY.itemsize
        L.check(L.lib().mcpt_shade(self.ctx, scene.handle, L.ptr(rays), L.ptr(hits), L.ptr(color), L.ptr(seeds), n,
                                   int(max_depth), _stream()))

    def accumulate(self, color, hist, count, max_attempt):
        """history.cl: running mean of non-zero samples."""
        n = count.numel()
        L.check(L.lib().mcpt_accumulate(self.ctx, L.ptr(color), L.ptr(hist), L.ptr(count), n, int(max_attempt),
                                        _stream()))

    def gamma_preview(self, color, out=None):
        """testkernel.cl func (ColorOut's GL display pass): float4 colours ->
        (pow(c, 1/2.2f) per channel, w = 0), a new float32 (n, 4) tensor unless
        `out` is given (may be `color` itself)."""
        if color.dtype != torch.float32 or not color.is_cuda or color.numel() % 4:
            raise L.MCPTError("gamma_preview: a float32 CUDA tensor of float4 colours")
        color = color.contiguous()
        if out is None:
            out = torch.empty_like(color)
        elif (out.dtype != torch.float32 or not out.is_cuda or out.device != color.device
              or not out.is_contiguous() or out.numel() != color.numel()):
            raise L.MCPTError("gamma_preview: out must be a contiguous float32 CUDA tensor the size of color")
        L.check(L.lib().mcpt_gamma_preview(self.ctx, L.ptr(color), L.ptr(out), color.numel() // 4, _stream()))
        return out.view(-1, 4)


def records(buf, dtype):
    """View a device byte buffer as host numpy records."""
    return buf.cpu().numpy().view(dtype)


def to_device(arr, device):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1)).to(device)


def build_hlbvh_device(tris, device=0):
    """HLBVH<CPU> built on the GPU (mcpt_build_hlbvh_device): the same 2n-1
    BVHNode records as scene.build_hlbvh.  `tris` is a host TRIANGLE array or a
    device byte tensor of them; returns a device byte tensor of the nodes."""
    if isinstance(tris, np.ndarray):
        n = len(tris)
        tris = to_device(tris, device)
    else:
        n = tris.numel() // L.TRIANGLE.itemsize
    if n == 0:
        raise ValueError("empty scene")
    nodes = torch.empty((2 * n - 1) * L.BVHNODE.itemsize, dtype=torch.uint8, device=tris.device)
    L.check(L.lib().mcpt_build_hlbvh_device(L.ptr(tris), n, L.ptr(nodes), _stream()))
    return nodes


def build_hlbvh_host_nodes(tris, device=0):
    """HLBVH<CPU> nodes built on the GPU and returned as a host BVHNODE array
    (bit-identical to scene.build_hlbvh; a `build` for SceneData.from_arrays)."""
    return records(build_hlbvh_device(tris, device), L.BVHNODE).copy()


def treelet_device(nodes, device=0):
    """TreeletBVH<CPU> (MCPT/BVH/treeletBVH.cpp:343-372, "bvhtype": "treelet")
    run on the GPU by mcpt_treelet_device.  `nodes` is a host BVHNODE array
    (returns a restructured host copy) or a device byte tensor (restructured
    in place and returned)."""
    host = isinstance(nodes, np.ndarray)
    d = to_device(nodes, device) if host else nodes
    n = d.numel() // L.BVHNODE.itemsize
    L.check(L.lib().mcpt_treelet_device(L.ptr(d), n, _stream()))
    return records(d, L.BVHNODE).copy() if host else d


def treelet_gpu_device(nodes, device=0):
    """TreeletBVH<GPU> (MCPT/BVH/treeletBVH.cpp:413-438, kernels/treeletBVH.cl),
    the tree every reference render traverses (scenebuild.cpp:87-95), run by
    mcpt_treelet_gpu_device.  `nodes` is a host BVHNODE array in the HLBVH
    layout (returns a restructured host copy) or a device byte tensor
    (restructured in place and returned)."""
    host = isinstance(nodes, np.ndarray)
    d = to_device(nodes, device) if host else nodes
    n = d.numel() // L.BVHNODE.itemsize
    L.check(L.lib().mcpt_treelet_gpu_device(L.ptr(d), n, _stream()))
    return records(d, L.BVHNODE).copy() if host else d
