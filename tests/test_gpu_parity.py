"""GPU parity: the HIP path (libmcpt_hip.so) against the reference's own OpenCL
kernels compiled for gfx950 (oracle/_ref, tests/refgpu.py) on the same inputs.

Bar: bit-exact.  Rays, hits, shade transitions, accumulated images, counts
and seed chains must match the reference kernels bit for bit.
Only Hit.triangle_id is exempt in the pruned mode: it is the reference's
"last accepted triangle" (objdef.h:262-265), which shade never reads; the
NOPRUNE mode reproduces it too.
"""
import functools

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402

from . import refgpu, scenes  # noqa: E402

needs_ref = pytest.mark.skipif(not refgpu.available(), reason="oracle/_ref not built (needs /root/reference at build time)")


@pytest.fixture(scope="module")
def rnd():
    return R.Renderer(0)


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def assert_bits_equal(a, b, what):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    same = bits(a) == bits(b)
    if not same.all():
        ia = np.nonzero(~same.reshape(len(a), -1).all(axis=1))[0]
        raise AssertionError("%s: %d / %d records differ, first %s\nmine=%r\nref =%r" % (
            what, len(ia), len(a), ia[:8], a[ia[:2]], b[ia[:2]]))


def ray_fields_equal(mine, ref, what):
    assert_bits_equal(mine["origin"], ref["origin"], what + ".origin")
    assert_bits_equal(mine["direction"], ref["direction"], what + ".direction")


def hit_fields_equal(mine, ref, live, what, check_tri=False):
    m, r = mine[live], ref[live]
    for f in ("t", "normal", "point", "material_id"):
        assert_bits_equal(m[f], r[f], what + "." + f)
    if check_tri:
        assert_bits_equal(m["triangle_id"], r["triangle_id"], what + ".triangle_id")


SCENES = [("cbox", scenes.cbox, scenes.CBOX_CAM), ("mis", scenes.mis, scenes.MIS_CAM),
          ("dining", scenes.dining, scenes.DINING_CAM)]


@needs_ref
@pytest.mark.parametrize("w,h", [(64, 48), (37, 21)])
@pytest.mark.parametrize("camjson", [scenes.CBOX_CAM, scenes.MIS_CAM, scenes.DINING_CAM])
def test_generate_rays_bitexact(rnd, camjson, w, h):
    cam = S.parse_camera(camjson)
    mine = R.records(rnd.generate_rays(cam, w, h), L.RAY)
    ref = refgpu.generate(cam, w, h)
    ray_fields_equal(mine, ref, "generateRay")


def _bounce_chain(rnd, data, camjson, w, h, depth, mode):
    """Run intersect+shade bounce by bounce on BOTH implementations, feeding
    each stage the reference's outputs, and compare every stage."""
    cam = S.parse_camera(camjson)
    dsc = rnd.upload(data)
    rays = refgpu.generate(cam, w, h)
    n = len(rays)
    seeds = R.default_seeds(n)
    colors = np.ones((n, 4), np.float32)
    hits = np.zeros(n, L.HIT)
    for b in range(depth):
        live = (rays["origin"][:, 3].view(np.int32) & np.int32(-16777216)) == 0
        ref_hits = refgpu.intersect(data, rays, hits=hits)
        mine_hits = R.records(rnd.intersect(dsc, R.to_device(rays, rnd.device), hits=R.to_device(hits, rnd.device),
                                            mode=mode), L.HIT)
        hit_fields_equal(mine_hits, ref_hits, live, "bounce%d.hit" % b, check_tri=(mode == L.MODE_NOPRUNE))
        hits = ref_hits
        r_rays, r_col, r_seed = refgpu.shade(data, rays, hits, colors, seeds, depth)
        d_rays = R.to_device(rays, rnd.device)
        d_col = torch.from_numpy(colors.copy()).to(rnd.device)
        d_seed = torch.from_numpy(seeds.view(np.int32).copy()).to(rnd.device)
        rnd.shade(dsc, d_rays, R.to_device(hits, rnd.device), d_col, d_seed, depth)
        m_rays = R.records(d_rays, L.RAY)
        assert_bits_equal(d_col.cpu().numpy(), r_col, "bounce%d.color" % b)
        assert_bits_equal(d_seed.cpu().numpy().view(np.uint32), r_seed, "bounce%d.seed" % b)
        ray_fields_equal(m_rays, r_rays, "bounce%d.ray" % b)
        rays, colors, seeds = r_rays, r_col, r_seed
    dsc.close()


@needs_ref
@pytest.mark.parametrize("mode", [L.MODE_EXACT, L.MODE_NOPRUNE])
@pytest.mark.parametrize("name,getter,camjson", SCENES)
def test_bounce_chain_bitexact(rnd, name, getter, camjson, mode):
    _bounce_chain(rnd, getter(), camjson, 48, 40, 6, mode)


@needs_ref
@pytest.mark.parametrize("max_attempt", [4, 16])
def test_accumulate_bitexact(rnd, max_attempt):
    w, h = 32, 16
    rng = np.random.default_rng(1)
    hist = np.zeros((w * h, 4), np.float32)
    count = np.zeros(w * h, np.int32)
    dh = torch.zeros((w * h, 4), dtype=torch.float32, device=rnd.device)
    dn = torch.zeros(w * h, dtype=torch.int32, device=rnd.device)
    for f in range(max_attempt + 3):
        col = rng.exponential(1.0, (w * h, 4)).astype(np.float32)
        col[rng.random(w * h) < 0.3] = 0.0
        col[:, 3] = 0.0
        rc, hist, count = refgpu.accumulate(col, hist, count, w, h, max_attempt)
        dc = torch.from_numpy(col).to(rnd.device)
        rnd.accumulate(dc, dh, dn, max_attempt)
        assert_bits_equal(dc.cpu().numpy(), rc, "display")
        assert_bits_equal(dh.cpu().numpy(), hist, "history")
        assert_bits_equal(dn.cpu().numpy(), count, "count")


def _render_both(rnd, data, camjson, w, h, depth, frames, attempt, mode=L.MODE_EXACT, **kw):
    cam = S.parse_camera(camjson)
    seeds = R.default_seeds(w * h)
    ref_hist, ref_count, ref_seeds = refgpu.render(data, cam, w, h, depth, frames, attempt, seeds)
    dsc = rnd.upload(data)
    st = rnd.new_state(w, h, seeds)
    rnd.render_frames(dsc, cam, st, depth, attempt, frames, mode=mode, **kw)
    torch.cuda.synchronize()
    out = st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()
    dsc.close()
    return out, (ref_hist, ref_count, ref_seeds)


@needs_ref
@pytest.mark.parametrize("name,getter,camjson,depth", [("cbox", scenes.cbox, scenes.CBOX_CAM, 4),
                                                       ("cbox_diffuse", scenes.cbox_diffuse, scenes.CBOX_CAM, 8),
                                                       ("mis", scenes.mis, scenes.MIS_CAM, 12),
                                                       ("dining", scenes.dining, scenes.DINING_CAM, 16)])
@pytest.mark.parametrize("schedule", [L.SCHED_SINGLE, L.SCHED_PAIRED])
def test_render_frames_bitexact(rnd, name, getter, camjson, depth, schedule):
    (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, getter(), camjson, 64, 64, depth, 6, 4, schedule=schedule)
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


@needs_ref
@pytest.mark.parametrize("name,getter,camjson,depth", [("cbox", scenes.cbox, scenes.CBOX_CAM, 4),
                                                       ("mis", scenes.mis, scenes.MIS_CAM, 12),
                                                       ("dining", scenes.dining, scenes.DINING_CAM, 16)])
@pytest.mark.parametrize("schedule", [L.SCHED_SINGLE, L.SCHED_PAIRED])
@pytest.mark.parametrize("quantized", [1, 2])
def test_render_node_formats_bitexact(rnd, name, getter, camjson, depth, schedule, quantized):
    """Both search-tree node formats, forced: the 64-B quantized nodes (decoded
    boxes strictly larger than the exact ones, the leaf's exact box re-tested
    in the L phase; auto-picked for trees beyond the L2) and the 128-B exact
    nodes match the reference kernels bit for bit."""
    rnd.set_tuning(quantized=quantized)
    try:
        (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, getter(), camjson, 64, 64, depth, 4, 4, schedule=schedule)
        assert rnd.stats()["quantized"] == (1 if quantized == 1 else 0)
    finally:
        rnd.set_tuning()
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


@needs_ref
def test_padded_leaf_boxes_keep_full_nodes_bitexact(rnd):
    """A tree whose leaf boxes are not the triangles' vertex bounds (a foreign
    BVH with padded leaves) cannot use the L phase's rebuilt leaf box: the scene
    keeps the 128-B nodes only, and still matches the reference kernels over the
    same padded tree."""
    data = scenes.cbox()
    nodes = data.nodes.copy()
    leaves = np.flatnonzero(nodes["left"] == nodes["right"])
    pad = leaves[::7]
    nodes["bbmin"][pad, :3] -= 0.25
    nodes["bbmax"][pad, :3] += 0.25
    # refit the internal boxes (unions again), so the tree stays a valid BVH
    order, stack = [], [0]
    while stack:
        k = stack.pop()
        order.append(k)
        if nodes["left"][k] != nodes["right"][k]:
            stack += [int(nodes["left"][k]), int(nodes["right"][k])]
    for k in reversed(order):
        l, r = nodes["left"][k], nodes["right"][k]
        if l != r:
            nodes["bbmin"][k] = np.minimum(nodes["bbmin"][l], nodes["bbmin"][r])
            nodes["bbmax"][k] = np.maximum(nodes["bbmax"][l], nodes["bbmax"][r])
    data = data.with_nodes(nodes)
    rnd.set_tuning(quantized=1)
    try:
        (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, data, scenes.CBOX_CAM, 64, 64, 6, 4, 4)
        assert rnd.stats()["quantized"] == 0
    finally:
        rnd.set_tuning()
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


@needs_ref
@pytest.mark.parametrize("name,getter,camjson,depth", [("cbox", scenes.cbox, scenes.CBOX_CAM, 6),
                                                       ("mis", scenes.mis, scenes.MIS_CAM, 12)])
def test_render_over_treelet_bvh_bitexact(rnd, name, getter, camjson, depth):
    """"bvhtype": "treelet": the restructured tree changes the reference's
    left-first visiting order (and so its tie winners); the HIP path over the
    same tree still matches the reference kernels bit for bit."""
    data = getter()
    data = data.with_nodes(R.treelet_device(data.nodes))
    _bounce_chain(rnd, data, camjson, 48, 40, 4, L.MODE_EXACT)
    (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, data, camjson, 64, 64, depth, 6, 4)
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


@needs_ref
@pytest.mark.parametrize("name,getter,camjson,depth", [("cbox", scenes.cbox, scenes.CBOX_CAM, 6),
                                                       ("mis", scenes.mis, scenes.MIS_CAM, 12),
                                                       ("dining", scenes.dining, scenes.DINING_CAM, 8)])
def test_render_over_gpu_treelet_bvh_bitexact(rnd, name, getter, camjson, depth):
    """The tree every reference render traverses (TreeletBVH<GPU>,
    scenebuild.cpp:87-95): the HIP path over mcpt_treelet_gpu_device's tree
    matches the reference kernels over the same tree bit for bit, per bounce
    and over whole renders."""
    data = getter()
    data = data.with_nodes(R.treelet_gpu_device(data.nodes))
    _bounce_chain(rnd, data, camjson, 48, 40, 4, L.MODE_EXACT)
    (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, data, camjson, 64, 64, depth, 6, 4)
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


NEAR_TIES = [("cbox", 0.0, scenes.CBOX_CAM), ("mis", 0.0, scenes.MIS_CAM), ("mis", 3e-6, scenes.MIS_CAM)]


@needs_ref
@pytest.mark.parametrize("name,offset,camjson", NEAR_TIES)
@pytest.mark.parametrize("quantized", [1, 2])
def test_near_ties_bitexact(rnd, name, offset, camjson, quantized):
    """Twin triangles less than EPS apart: the nearest-first search must hand
    these rays to the reference-order search and still match bit for bit
    (with either search-tree node format)."""
    data = scenes.near_ties(name, offset)
    _bounce_chain(rnd, data, camjson, 48, 40, 4, L.MODE_EXACT)
    rnd.set_stats(True)
    rnd.set_tuning(quantized=quantized)
    try:
        (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, data, camjson, 64, 64, 6, 4, 4)
        fallbacks = rnd.stats()["order_fallbacks"]
    finally:
        rnd.set_stats(False)
        rnd.set_tuning()
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")
    assert fallbacks > 0


@needs_ref
def test_render_frames_chunked_and_striped_bitexact(rnd):
    """Frames split across launches and rows split into stripes (the multi-GPU
    partition, run sequentially here) change nothing."""
    data, cam = scenes.cbox(), S.parse_camera(scenes.CBOX_CAM)
    w, h, depth, frames, attempt = 48, 40, 5, 7, 4
    seeds = R.default_seeds(w * h)
    rh, rc, rs = refgpu.render(data, cam, w, h, depth, frames, attempt, seeds)
    dsc = rnd.upload(data)
    for stripes in (1, 3):
        st = rnd.new_state(w, h, seeds)
        for k in range(stripes):
            for f0, nf in ((0, 2), (2, 5)):
                rnd.render_frames(dsc, cam, st, depth, attempt, nf, frame_begin=f0, stripe_rows=8, stripe_index=k,
                                  stripe_count=stripes, frames_per_launch=3)
        torch.cuda.synchronize()
        assert_bits_equal(st.count.cpu().numpy(), rc, "count/%d" % stripes)
        assert_bits_equal(st.seeds_np(), rs, "seeds/%d" % stripes)
        assert_bits_equal(st.hist.cpu().numpy(), rh, "hist/%d" % stripes)
    dsc.close()


@needs_ref
@pytest.mark.parametrize("cache", [2, 1])
def test_orthographic_camera_render_bitexact(rnd, cache):
    """rayGenerator.cl's second camera (camera_type 1: every ray along the view
    direction, origins spread over the image plane; parseCamera never makes it,
    a C host can).  A frame started from the primary-hit record takes the
    per-pixel origin from the record and the shared direction from the launch:
    the reference's bits, cache off and on."""
    data = scenes.mis()
    cam = S.parse_camera(scenes.MIS_CAM).copy()
    cam["camera_type"] = 1
    cam["arg"] = np.float32(9.5)  # the image plane's width in scene units
    w, h, depth, frames, attempt = 40, 32, 6, 4, 8
    seeds = R.default_seeds(w * h)
    rh, rc, rs = refgpu.render(data, cam, w, h, depth, frames, attempt, seeds)
    dsc = rnd.upload(data)
    try:
        rnd.set_tuning(primary_cache=cache)
        st = rnd.new_state(w, h, seeds)
        rnd.render_frames(dsc, cam, st, depth, attempt, frames)
        assert rnd.stats()["primary_cache"] == (2 if cache == 1 else 0)
        torch.cuda.synchronize()
        assert_bits_equal(st.count.cpu().numpy(), rc, "count")
        assert_bits_equal(st.seeds_np(), rs, "seeds")
        assert_bits_equal(st.hist.cpu().numpy(), rh, "hist")
        assert (rc > 0).mean() > 0.05  # some rays reach lit surfaces (measured 0.13)
    finally:
        rnd.set_tuning()
        dsc.close()


@needs_ref
@pytest.mark.parametrize("mode", [L.MODE_EXACT, L.MODE_NOPRUNE])
@pytest.mark.parametrize("name,getter,camjson", [("cbox", scenes.cbox, scenes.CBOX_CAM), ("mis", scenes.mis, scenes.MIS_CAM)])
def test_primary_hit_cache_bitexact(rnd, name, getter, camjson, mode):
    """Every frame re-shoots the same primary ray (rayGenerator.cl has no
    jitter), so k_render reads each pixel's primary hit from a cache computed
    once per (scene, camera, image, stripes, mode).  Off, always, and auto
    across split calls: the reference's bits every time, and the cache is
    computed, reused and invalidated when it should be."""
    data, cam = getter(), S.parse_camera(camjson)
    w, h, depth, frames, attempt = 48, 40, 6, 5, 8
    seeds = R.default_seeds(w * h)
    rh, rc, rs = refgpu.render(data, cam, w, h, depth, frames, attempt, seeds)
    dsc = rnd.upload(data)

    def check(st, what):
        torch.cuda.synchronize()
        assert_bits_equal(st.count.cpu().numpy(), rc, what + "/count")
        assert_bits_equal(st.seeds_np(), rs, what + "/seeds")
        assert_bits_equal(st.hist.cpu().numpy(), rh, what + "/hist")

    try:
        for pc, want in ((2, 0), (1, 2)):
            rnd.set_tuning(primary_cache=pc)
            st = rnd.new_state(w, h, seeds)
            rnd.render_frames(dsc, cam, st, depth, attempt, frames, mode=mode)
            assert rnd.stats()["primary_cache"] == want
            check(st, "primary_cache=%d" % pc)
        rnd.set_tuning()
        dsc2 = rnd.upload(data)  # a new scene: the cache of dsc no longer applies
        st = rnd.new_state(w, h, seeds)
        rnd.render_frames(dsc2, cam, st, depth, attempt, 1, mode=mode)
        assert rnd.stats()["primary_cache"] == 0  # a one-frame call does not build it
        rnd.render_frames(dsc2, cam, st, depth, attempt, 2, mode=mode)
        assert rnd.stats()["primary_cache"] == 2  # built
        rnd.render_frames(dsc2, cam, st, depth, attempt, 1, mode=mode)
        assert rnd.stats()["primary_cache"] == 1  # reused, one frame too
        rnd.render_frames(dsc2, cam, st, depth, attempt, 1, mode=mode)
        check(st, "auto, split calls")
        other = cam.copy()
        other.view(np.float32)[0] += np.float32(0.25)  # another camera
        st2 = rnd.new_state(w, h, seeds)
        rnd.render_frames(dsc2, other, st2, depth, attempt, 1, mode=mode)
        assert rnd.stats()["primary_cache"] == 0  # a new view, one frame: traced
        rnd.render_frames(dsc2, other, st2, depth, attempt, 1, mode=mode)
        assert rnd.stats()["primary_cache"] == 2  # the same view again: built
        rnd.render_frames(dsc2, cam, st2, depth, attempt, 2, mode=mode)
        assert rnd.stats()["primary_cache"] == 2  # back to the first camera: rebuilt
        dsc2.close()
    finally:
        rnd.set_tuning()
    dsc.close()


def test_exact_equals_noprune_full_size(rnd):
    """Size-independent property at a C2-like configuration: the pruned
    traversal reproduces the exhaustive reference traversal exactly."""
    data, cam = scenes.cbox_diffuse(), S.parse_camera(scenes.CBOX_CAM)
    w = h = 256
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    outs = []
    for mode in (L.MODE_EXACT, L.MODE_NOPRUNE):
        st = rnd.new_state(w, h, seeds)
        rnd.render_frames(dsc, cam, st, 8, 256, 4, mode=mode)
        torch.cuda.synchronize()
        outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
    for a, b, what in zip(outs[0], outs[1], ("hist", "count", "seeds")):
        assert_bits_equal(a, b, what)
    dsc.close()


def test_launch_knobs_change_no_bits_full_size(rnd):
    """Size-independent property at a C2-like configuration: every launch-plan
    knob Renderer.tune and bench.py set (S-phase and fetch thresholds, leaf
    threshold, queue chunk, block sizing, queue count, the dearest-first tile
    order) moves only speed: the image, counts and seed chains are identical
    for each setting."""
    data, cam = scenes.cbox_diffuse(), S.parse_camera(scenes.CBOX_CAM)
    w = h = 256
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    settings = [{}, {"shade_threshold": 48, "fetch_threshold": 8}, {"shade_threshold": 24, "leaf_threshold": 8},
                {"fetch_threshold": 64, "queue_chunk": 16}, {"block_entries": 4, "max_block_frames": 2},
                {"queues": 1}, {"queues": 3, "fetch_threshold": 5}, {"primary_cache": 2}, {"primary_cache": 1},
                {"tile_order": 1}, {"tile_order": 2}, {"tile_order": 2, "queues": 3}, {"pixel_spread": 2},
                {"pixel_spread": 2, "queues": 3, "block_entries": 4, "max_block_frames": 2},
                {"pixel_spread": 2, "tile_order": 1, "queues": 5}]
    outs = []
    try:
        for t in settings:
            rnd.set_tuning(**t)
            st = rnd.new_state(w, h, seeds)
            rnd.render_frames(dsc, cam, st, 8, 1 << 20, 6)
            torch.cuda.synchronize()
            outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
    finally:
        rnd.set_tuning()
    for t, o in zip(settings[1:], outs[1:]):
        for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
            assert_bits_equal(a, b, "%s %s" % (what, t))
    dsc.close()


@pytest.mark.parametrize("wh", [(100, 75), (8, 8), (520, 9)])
def test_pixel_spread_ragged_images(rnd, wh):
    """The spread slot mapping (mcpt_tuning.pixel_spread 2: a wave's 64
    consecutive queue slots are one pixel of each of up to 64 tiles) is a
    bijection on every queue's slots, partial last groups and edge-tile holes
    included: ragged images render every pixel exactly as tile-major slots do,
    with one block per pixel and with several."""
    data, cam = scenes.cbox_diffuse(), S.parse_camera(scenes.CBOX_CAM)
    w, h = wh
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    outs = []
    try:
        for t in ({"pixel_spread": 1}, {"pixel_spread": 2}, {"pixel_spread": 2, "queues": 3},
                  {"pixel_spread": 2, "block_entries": 64, "max_block_frames": 1}):
            rnd.set_tuning(**t)
            st = rnd.new_state(w, h, seeds)
            rnd.render_frames(dsc, cam, st, 6, 1 << 20, 5)
            torch.cuda.synchronize()
            outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
    finally:
        rnd.set_tuning()
    for o in outs[1:]:
        for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
            assert_bits_equal(a, b, what)
    dsc.close()


def test_frame_blocks_handoff_full_size(rnd):
    """Frame blocks of one pixel run on different lanes (and XCDs) within one
    launch, handing the state through memory: any block size gives the same
    bits as one block per pixel."""
    data, cam = scenes.cbox_diffuse(), S.parse_camera(scenes.CBOX_CAM)
    w = h = 512
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    outs = []
    for fpl in (24, 1, 5):
        st = rnd.new_state(w, h, seeds)
        rnd.render_frames(dsc, cam, st, 8, 1 << 20, 24, frames_per_launch=fpl)
        torch.cuda.synchronize()
        outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
    for o in outs[1:]:
        for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
            assert_bits_equal(a, b, what)
    dsc.close()


@pytest.mark.parametrize("diffuse", [True, False])
def test_short_last_block_same_bits(rnd, diffuse):
    """mcpt_tuning.last_block_frames: on an image with several pixels per
    resident lane the auto plan's blocks become (long head blocks, one short
    last block); the frame range each block covers and the MAX_ATTEMPT cut
    inside the last block give the same bits as one block per pixel."""
    data = scenes.cbox_diffuse() if diffuse else scenes.cbox()
    cam = S.parse_camera(scenes.CBOX_CAM)
    w = h = 1024
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    try:
        for attempt in (1 << 20, 18):
            outs, fpbs = [], []
            for t, fpl in (({}, 20), ({"last_block_frames": -1}, 0), ({"last_block_frames": 2}, 0),
                           ({"last_block_frames": 3, "block_entries": 12}, 0), ({"last_block_frames": 9}, 0),
                           ({}, 0)):
                rnd.set_tuning(**t)
                st = rnd.new_state(w, h, seeds)
                rnd.render_frames(dsc, cam, st, 8, attempt, 20, frames_per_launch=fpl)
                torch.cuda.synchronize()
                fpbs.append(rnd.stats()["frames_per_block"])
                outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
            assert fpbs[0] == 20 and fpbs[2] == 18, fpbs  # (18, 2): the short last block did run
            # the auto plan's regime follows the pixels per resident lane (the
            # grid is the resident capacity): between 2.5 and 6 on a whole image
            # it is (15, 5), a last block of ceil(20 / 4) (gfx950 today: 4 per lane)
            ppl = float(w * h) / (rnd.stats()["workgroups"] * 64)
            if 2.5 < ppl < 6.0:
                assert fpbs[5] == 15, (fpbs, ppl)
            for o in outs[1:]:
                for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
                    assert_bits_equal(a, b, what)
        # 64 frames (Renderer.tune's default call): 2 auto blocks of 32; a last
        # block of 8 would need a 56-frame head block, above the 32-frame cap,
        # so the plan keeps equal blocks (no block exceeds the cap)
        outs, fpbs = [], []
        for t, fpl in (({}, 64), ({"last_block_frames": 8}, 0), ({"last_block_frames": 20}, 0)):
            rnd.set_tuning(**t)
            st = rnd.new_state(w, h, seeds)
            rnd.render_frames(dsc, cam, st, 8, 1 << 20, 64, frames_per_launch=fpl)
            torch.cuda.synchronize()
            fpbs.append(rnd.stats()["frames_per_block"])
            outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
        assert fpbs[0] == 64 and all(f <= 32 for f in fpbs[1:]), fpbs
        for o in outs[1:]:
            for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
                assert_bits_equal(a, b, what)
    finally:
        rnd.set_tuning()
        dsc.close()


def test_image_beyond_handoff_range(rnd):
    """The block hand-off addresses its per-pixel granules with 32-bit byte
    offsets below 2^31 (67 M pixels); a larger image runs one block per pixel
    per launch whatever frames_per_launch asks, so it completes, and with the
    same bits as one explicit block; each launch runs at most max_block_frames
    frames (VERDICT/ADVICE r3: a whole call in one dispatch was unbounded)."""
    data, cam = scenes.cbox_diffuse(), S.parse_camera(scenes.CBOX_CAM)
    w, h = 8192, 8200
    assert w * h * 32 > 2 ** 31
    dsc = rnd.upload(data)
    seeds = R.default_seeds(w * h)
    outs = []
    try:
        # (frames_per_launch, max_block_frames) -> launches: one block per
        # launch, every launch at most the block cap's frames (5 frames at a
        # cap of 2: blocks 2, 2, 1, chained through the state arrays)
        for (fpl, capf), want in (((1, 0), 5), ((5, 0), 1), ((0, 2), 3), ((4, 2), 3)):
            rnd.set_tuning(max_block_frames=capf)
            st = rnd.new_state(w, h, seeds)
            rnd.render_frames(dsc, cam, st, 2, 1 << 20, 5, frames_per_launch=fpl)
            torch.cuda.synchronize()
            assert rnd.stats()["launches"] == want, (fpl, capf, rnd.stats()["launches"])
            outs.append(st)
        for o in outs[1:]:
            assert torch.equal(outs[0].hist, o.hist) and torch.equal(outs[0].count, o.count)
            assert torch.equal(outs[0].seeds, o.seeds)
        assert int((outs[0].count > 0).sum()) > w * h // 100  # depth 2: 1.7 % of the paths reach the light
    finally:
        rnd.set_tuning()
        del outs
        dsc.close()


@needs_ref
@pytest.mark.parametrize("name,getter,camjson,depth", [("cbox", scenes.cbox, scenes.CBOX_CAM, 8),
                                                       ("dining", scenes.dining, scenes.DINING_CAM, 16)])
@pytest.mark.parametrize("schedule", [L.SCHED_SINGLE, L.SCHED_PAIRED])
@pytest.mark.parametrize("quantized", [1, 2])
def test_render_windowed_stack_bitexact(rnd, name, getter, camjson, depth, schedule, quantized):
    """The LDS-window stack (top 32 entries in LDS, the rest spilled to a
    per-lane global area; picked at launch for deep trees) is the same
    logical stack: forced on, renders still match the reference bit for bit."""
    rnd.set_tuning(stack_window=1, quantized=quantized)
    try:
        (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, getter(), camjson, 64, 64, depth, 4, 4, schedule=schedule)
    finally:
        rnd.set_tuning()
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


@pytest.mark.parametrize("mode", [L.MODE_EXACT, L.MODE_NOPRUNE])
def test_paired_schedule_equals_single_full_size(rnd, mode):
    """Size-independent property at the C2 and C3 configurations: the paired
    leaf-test schedule (MCPT_SCHED_PAIRED) changes only speed, never bits."""
    for getter, camjson, depth, w in ((scenes.cbox_diffuse, scenes.CBOX_CAM, 8, 512),
                                      (scenes.mis, scenes.MIS_CAM, 12, 384)):
        data, cam = getter(), S.parse_camera(camjson)
        seeds = R.default_seeds(w * w)
        dsc = rnd.upload(data)
        outs = []
        for sched in (L.SCHED_SINGLE, L.SCHED_PAIRED):
            st = rnd.new_state(w, w, seeds)
            rnd.render_frames(dsc, cam, st, depth, 1 << 20, 8, mode=mode, schedule=sched)
            torch.cuda.synchronize()
            outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
        for a, b, what in zip(outs[0], outs[1], ("hist", "count", "seeds")):
            assert_bits_equal(a, b, what)
        dsc.close()


def test_tune_schedule_leaves_state_alone(rnd):
    """Renderer.tune_schedule renders on a scratch copy: the caller's state is
    untouched, the scene keeps a valid schedule, and rendering afterwards
    gives the untuned bits."""
    data, cam = scenes.mis(), S.parse_camera(scenes.MIS_CAM)
    w = h = 128
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    ref = rnd.new_state(w, h, seeds)
    rnd.render_frames(dsc, cam, ref, 12, 1 << 20, 6, schedule=L.SCHED_SINGLE)
    st = rnd.new_state(w, h, seeds)
    sched, best = rnd.tune_schedule(dsc, cam, st, 12, 1 << 20, frames=4, trials=1)
    assert sched in (L.SCHED_SINGLE, L.SCHED_PAIRED) and dsc.schedule == sched
    assert set(best) == {L.SCHED_SINGLE, L.SCHED_PAIRED} and all(v > 0 for v in best.values())
    assert st.frames_done == 0 and int(st.count.sum()) == 0 and float(st.hist.abs().sum()) == 0.0
    assert_bits_equal(st.seeds_np(), seeds.astype(np.uint32), "seeds untouched")
    rnd.render_frames(dsc, cam, st, 12, 1 << 20, 6)
    torch.cuda.synchronize()
    for a, b, what in zip((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()),
                          (ref.hist.cpu().numpy(), ref.count.cpu().numpy(), ref.seeds_np()), ("hist", "count", "seeds")):
        assert_bits_equal(a, b, what)
    with pytest.raises(L.MCPTError):
        rnd.render_frames(dsc, cam, st, 12, 1 << 20, 1, schedule=7)
    # the combined tuning (schedule x S-phase threshold) leaves the state alone too
    st2 = rnd.new_state(w, h, seeds)
    sched, th, best2 = rnd.tune(dsc, cam, st2, 12, 1 << 20, frames=4, trials=1)
    try:
        assert th in (32, 40, 48) and rnd.get_tuning()["shade_threshold"] == th and dsc.schedule == sched
        # 3 S thresholds x 2 schedules, the other fetch threshold, the other 5 (block sizing, tile
        # order) pairs, and the other two S thresholds again when that pair changed
        assert len(best2) in (12, 14) and int(st2.count.sum()) == 0
        assert (rnd.get_tuning()["block_entries"] or 8) in (8, 16)
        assert rnd.get_tuning()["tile_order"] in (0, 1, 2)
        assert rnd.get_tuning()["last_block_frames"] in (-1, 0, 1)  # equal, auto, ceil(4 / 8) or ceil(4 / 4)
        rnd.render_frames(dsc, cam, st2, 12, 1 << 20, 6)
        torch.cuda.synchronize()
        assert_bits_equal(st2.hist.cpu().numpy(), ref.hist.cpu().numpy(), "hist after tune")
        assert_bits_equal(st2.seeds_np(), ref.seeds_np(), "seeds after tune")
    finally:
        rnd.set_tuning()
    dsc.close()


@needs_ref
@pytest.mark.parametrize("w,h,depth,frames,attempt", [(1, 1, 4, 5, 4), (7, 3, 6, 9, 2), (65, 33, 3, 4, 0),
                                                      (130, 9, 1, 3, 8)])
@pytest.mark.parametrize("schedule", [L.SCHED_SINGLE, L.SCHED_PAIRED])
def test_render_edge_sizes_bitexact(rnd, w, h, depth, frames, attempt, schedule):
    """Ragged and tiny images (edge tiles with holes, a 1x1 image), depth 1,
    and the MAX_ATTEMPT cap at 0 (history never runs) match the reference."""
    (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, scenes.cbox(), scenes.CBOX_CAM, w, h, depth, frames, attempt,
                                              schedule=schedule, frames_per_launch=2)
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


@functools.lru_cache(None)
def _c5_small():
    """C5's scene family (BASELINE.json configs[4], scene.random_mesh) at
    500 K triangles: a deep random-soup HLBVH."""
    return S.random_mesh(500_000, seed=7)


@needs_ref
@pytest.mark.parametrize("schedule", [L.SCHED_SINGLE, L.SCHED_PAIRED])
@pytest.mark.parametrize("quantized", [1, 2])
def test_random_mesh_c5_bitexact(rnd, schedule, quantized):
    """C5 (the deep-BVH random mesh): 500 K triangles at 64x64, depth 8, 5
    frames, the stack layout on auto (picked by the occupancy rule, not
    forced), the frames in 2-frame blocks handed between lanes.
    The reference's own kernels traverse the same tree with their fixed
    int stack[64] (objdef.h:247); images, counts and seeds match bit for
    bit."""
    data = _c5_small()
    assert S.bvh_stack_depth(data.nodes) <= 64  # within the reference's stack
    rnd.set_tuning(quantized=quantized)
    try:
        (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, data, S.RANDOM_MESH_CAMERA, 64, 64, 8, 5, 4, schedule=schedule,
                                                  frames_per_launch=2)
        st = rnd.stats()
    finally:
        rnd.set_tuning()
    assert st["quantized"] == (1 if quantized == 1 else 0)
    assert st["frames_per_block"] == 2 and st["stack_window"] in (0, 1)  # 3 blocks: hand-offs happened
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")
    assert (rc > 0).any()  # the light is seen through the soup


def test_random_mesh_c5_full_size_properties(rnd):
    """C5 at its full size: 10 M random triangles, the HLBVH built on the GPU
    (mcpt_build_hlbvh_device), 2048x2048, depth 8, 2 frames.  Size-independent
    properties: one 2-frame block (the auto plan: the quantized search tree,
    this tree being far beyond the L2), two 1-frame blocks handed between
    lanes, the rows split into 3 GPUs' stripes rendered in turn, and the
    128-B exact nodes give the same bits; radiance is finite and
    non-negative, counts are within [0, 2] and some pixels see the light."""
    data = S.random_mesh(10_000_000, build=R.build_hlbvh_host_nodes)
    cam = S.parse_camera(S.RANDOM_MESH_CAMERA)
    w = h = 2048
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    outs = []
    for stripes, fpl, quantized in ((1, 2, 0), (1, 1, 0), (3, 1, 0), (1, 2, 2)):
        st = rnd.new_state(w, h, seeds)
        rnd.set_tuning(quantized=quantized)
        try:
            for k in range(stripes):
                rnd.render_frames(dsc, cam, st, 8, 1 << 20, 2, stripe_rows=16, stripe_index=k, stripe_count=stripes,
                                  frames_per_launch=fpl)
            torch.cuda.synchronize()
            assert rnd.stats()["quantized"] == (1 if quantized == 0 else 0)
        finally:
            rnd.set_tuning()
        outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
    dsc.close()
    for o in outs[1:]:
        for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
            assert_bits_equal(a, b, what)
    hist, count = outs[0][0], outs[0][1]
    assert np.isfinite(hist).all() and (hist >= 0).all()
    assert count.min() >= 0 and count.max() <= 2 and (count > 0).sum() > 1000


def test_render_zero_frames_and_bad_params(rnd):
    """frames = 0 is a no-op; malformed parameters are status errors."""
    data, cam = scenes.cbox(), S.parse_camera(scenes.CBOX_CAM)
    w = h = 16
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    st = rnd.new_state(w, h, seeds)
    rnd.render_frames(dsc, cam, st, 4, 4, 0)
    torch.cuda.synchronize()
    assert int(st.count.sum()) == 0 and float(st.hist.abs().sum()) == 0.0
    assert_bits_equal(st.seeds_np(), seeds.astype(np.uint32), "seeds")
    for kw in (dict(stripe_index=2, stripe_count=2), dict(stripe_rows=0), dict(mode=5)):
        with pytest.raises(L.MCPTError):
            rnd.render_frames(dsc, cam, st, 4, 4, 1, **kw)
    with pytest.raises(L.MCPTError):
        rnd.render_frames(dsc, cam, st, 0, 4, 1)  # max_depth must be >= 1
    with pytest.raises(L.MCPTError):
        rnd.render_frames(dsc, cam, st, 4, 4, -1)
    with pytest.raises(L.MCPTError):
        rnd.set_tuning(last_block_frames=-2)  # -1 equal blocks, 0 auto, > 0 frames
    dsc.close()


def test_handoff_tag_wrap_bitexact(rnd):
    """Block hand-off tags carry 8 bits of launch sequence: after 255 launches
    they wrap and mcpt_render_frames clears the granule area first.  300 calls
    of two one-frame blocks (one hand-off per pixel each) cross the wrap; the
    image equals one 600-frame call's (255 blocks per launch: 3 launches) and
    the reference kernels' bit for bit."""
    data, cam = scenes.cbox(), S.parse_camera(scenes.CBOX_CAM)
    w, h, depth = 24, 16, 4
    seeds = R.default_seeds(w * h, variant="msvc15")
    dsc = rnd.upload(data)
    att = 1024  # a MAX_ATTEMPT the reference's history kernel is built for (oracle/Makefile)
    a = rnd.new_state(w, h, seeds)
    for _ in range(300):
        rnd.render_frames(dsc, cam, a, depth, att, 2, frames_per_launch=1)
        assert rnd.stats()["frames_per_block"] == 1
    b = rnd.new_state(w, h, seeds)
    rnd.render_frames(dsc, cam, b, depth, att, 600, frames_per_launch=1)
    assert rnd.stats()["launches"] == 3
    for x, y, what in ((a.hist, b.hist, "hist"), (a.count, b.count, "count"), (a.seeds, b.seeds, "seeds")):
        assert_bits_equal(x.cpu().numpy(), y.cpu().numpy(), what)
    if refgpu.available():
        rh, rc, rs = refgpu.render(data, cam, w, h, depth, 600, att, seeds)
        assert_bits_equal(b.hist.cpu().numpy(), rh, "hist vs reference")
        assert_bits_equal(b.seeds_np(), rs, "seeds vs reference")
    dsc.close()


@needs_ref
@pytest.mark.parametrize("name,getter,camjson,depth", [("cbox", scenes.cbox, scenes.CBOX_CAM, 6),
                                                       ("mis", scenes.mis, scenes.MIS_CAM, 12),
                                                       ("dining", scenes.dining, scenes.DINING_CAM, 16)])
@pytest.mark.parametrize("levels", [-1, 1, 2, 3, 4, "max"])
@pytest.mark.parametrize("quantized", [1, 2])
def test_top_levels_bitexact(rnd, name, getter, camjson, depth, levels, quantized):
    """The search tree's top levels in LDS (mcpt_tuning.top_levels: none, 1, 2
    3 or 4 levels descended where a segment begins, from the exact 128-B nodes
    also for the quantized tree; 4 needs several waves per workgroup,
    MCPT_WG_WAVES, as shipped): every setting matches the reference kernels
    bit for bit, with either node format."""
    # "max": the most this build keeps (MCPT_WG_WAVES: 1 wave 3, 2-4 waves 4 as
    # shipped, 8 waves 5: `make variants` builds under MCPT_LIB_OVERRIDE)
    levels = _max_top_levels(rnd) if levels == "max" else levels
    try:
        rnd.set_tuning(top_levels=levels, quantized=quantized)
    except L.MCPTError:
        assert levels == 4
        pytest.skip("a one-wave-per-workgroup variant build keeps at most 3 levels")
    try:
        (h_, c_, s_), (rh, rc, rs) = _render_both(rnd, getter(), camjson, 64, 64, depth, 4, 4)
        st = rnd.stats()
    finally:
        rnd.set_tuning()
    assert st["top_levels"] == (0 if levels < 0 else levels) and st["quantized"] == (1 if quantized == 1 else 0)
    assert_bits_equal(c_, rc, "count")
    assert_bits_equal(s_, rs, "seeds")
    assert_bits_equal(h_, rh, "hist")


def _max_top_levels(rnd):
    """The most top levels this build keeps (MCPT_WG_WAVES: 3, 4 or 5)."""
    for k in (5, 4):
        try:
            rnd.set_tuning(top_levels=k)
            return k
        except L.MCPTError:
            pass
        finally:
            rnd.set_tuning()
    return 3


def test_top_levels_full_size_same_bits(rnd):
    """Size-independent property at C2's and C4's sizes: every top_levels
    setting gives the same image, on the whole image and on an 8-rank share;
    auto takes 2 levels on cbox (2.1 MB tree) and the build's most (4 as
    shipped) on the dining proxy."""
    deep = _max_top_levels(rnd)
    for getter, camjson, depth, w, h, frames, auto in ((scenes.cbox_diffuse, scenes.CBOX_CAM, 8, 1024, 1024, 6, 2),
                                                       (scenes.dining, scenes.DINING_CAM, 16, 1920, 1080, 2, deep)):
        data, cam = getter(), S.parse_camera(camjson)
        seeds = R.default_seeds(w * h)
        dsc = rnd.upload(data)
        try:
            for stripes in (1, 8):
                outs = []
                for levels in (-1, 0, 3):
                    rnd.set_tuning(top_levels=levels)
                    st = rnd.new_state(w, h, seeds)
                    rnd.render_frames(dsc, cam, st, depth, 1 << 30, frames, stripe_rows=16, stripe_index=stripes - 1,
                                      stripe_count=stripes)
                    torch.cuda.synchronize()
                    assert rnd.stats()["top_levels"] == {-1: 0, 0: auto, 3: 3}[levels]
                    outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
                for o in outs[1:]:
                    for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
                        assert_bits_equal(a, b, "%s / %d stripes" % (what, stripes))
        finally:
            rnd.set_tuning()
            dsc.close()
