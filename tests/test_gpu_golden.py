"""GPU parity against the COMMITTED reference outputs (tests/golden/, produced
by the reference's own kernels on an MI355X, tools/make_goldens.py): runs even
where oracle/_ref is not built.  Bar: bit-exact.  Plus full-size properties
and a statistical check against the CPU oracle."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402

from . import oracle as O  # noqa: E402
from . import scenes  # noqa: E402
from .test_gpu_parity import assert_bits_equal, ray_fields_equal  # noqa: E402

GOLD = os.path.join(scenes.ROOT, "tests", "golden")
CAMS = {"cbox": scenes.CBOX_CAM, "mis": scenes.MIS_CAM, "dining": scenes.DINING_CAM}


def gold(n):
    return np.load(os.path.join(GOLD, n))


@pytest.fixture(scope="module")
def rnd():
    return R.Renderer(0)


def test_inline_sincos_matches_ocml(rnd):
    # all 32768 randomDirection angles and every float in [0, 8), bit for bit
    assert rnd.selfcheck_trig() == (0, 0)


def test_lobe_pow_matches_ocml(rnd):
    """shade.cl:139's pow(cos_r, Ns) restated without ocml's special cases
    (cl_pow_lobe): every float in (0, 1 + 2^-10] for every glossy exponent of
    the scenes (cbox, veach_mis, the dining proxy) and edge exponents gives
    __ocml_pow_f32's bits."""
    from . import scenes
    ns = set()
    for getter in (scenes.cbox, scenes.mis, scenes.dining):
        m = getter().mats
        ns |= {float(x) for x in m["Ns"][m["type"] == L.MCPT_GLOSSY]}
    assert len(ns) >= 4  # veach_mis alone has four plates
    edges = [0.0, 1e-3, 0.5, 1.0, 2.0, 3.5, 7.25, 50.0, 100.0, 500.0, 4000.0, 65536.0]
    assert rnd.selfcheck_pow(sorted(ns) + edges) == 0


def test_lobe_pow_matches_ocml_exponent_sweep(rnd):
    """The restatement's whole exponent domain, not only the scenes' Ns: a
    stratified seeded sweep of y over [0, 65536] (log-uniform over 2^-20..2^16,
    uniform over [0, 65536], integers and half-integers, the domain's top
    floats), every float x in (0, 1 + 2^-10] for each: __ocml_pow_f32's bits.
    A user scene's Ns outside the tested list is covered by the domain
    argument of mcpt_refmath.h:121-130 and this sweep together."""
    g = np.random.default_rng(20261018)
    ys = list(np.float32(2.0) ** g.uniform(-20.0, 16.0, 24).astype(np.float32))
    ys += list(g.uniform(0.0, 65536.0, 12).astype(np.float32))
    ys += [float(v) for v in g.integers(1, 65536, 8)] + [float(v) + 0.5 for v in g.integers(1, 65535, 4)]
    ys += [float(np.nextafter(np.float32(65536.0), np.float32(0.0))), 65535.0, 1.0e-30, 3.0]
    ys = sorted({float(np.float32(y)) for y in ys})
    assert all(0.0 <= y <= 65536.0 for y in ys) and len(ys) >= 48
    assert rnd.selfcheck_pow(ys) == 0


@pytest.mark.parametrize("k", list(CAMS))
def test_rays_equal_golden(rnd, k):
    mine = R.records(rnd.generate_rays(S.parse_camera(CAMS[k]), 64, 48), L.RAY)
    ray_fields_equal(mine, gold("rays.npz")[k].view(L.RAY), "rays/" + k)


@pytest.mark.parametrize("name", ["cbox", "mis"])
@pytest.mark.parametrize("mode", [L.MODE_EXACT, L.MODE_NOPRUNE])
def test_bounce_chain_equals_golden(rnd, name, mode):
    c = gold("chain_%s.npz" % name)
    data = scenes.cbox() if name == "cbox" else scenes.mis()
    dsc = rnd.upload(data)
    depth = int(c["depth"])
    for b in range(depth):
        rays = c["rays%d" % b].view(L.RAY)
        href = c["hits%d" % b].view(L.HIT)
        live = (rays["origin"][:, 3].view(np.int32) & np.int32(-16777216)) == 0
        h = R.records(rnd.intersect(dsc, R.to_device(rays, rnd.device),
                                    hits=R.to_device(c["hits_in%d" % b].view(L.HIT), rnd.device), mode=mode), L.HIT)
        for f in ("t", "normal", "point", "material_id"):
            assert_bits_equal(h[f][live], href[f][live], "b%d.%s" % (b, f))
        if mode == L.MODE_NOPRUNE:
            assert_bits_equal(h["triangle_id"][live], href["triangle_id"][live], "b%d.tri" % b)
        d_rays = R.to_device(rays, rnd.device)
        d_col = torch.from_numpy(c["colors_in%d" % b].copy()).to(rnd.device)
        d_seed = torch.from_numpy(c["seeds_in%d" % b].view(np.int32).copy()).to(rnd.device)
        rnd.shade(dsc, d_rays, R.to_device(href, rnd.device), d_col, d_seed, depth)
        assert_bits_equal(d_col.cpu().numpy(), c["colors%d" % b], "b%d.color" % b)
        assert_bits_equal(d_seed.cpu().numpy().view(np.uint32), c["seeds%d" % b], "b%d.seed" % b)
        ray_fields_equal(R.records(d_rays, L.RAY), c["rays_out%d" % b].view(L.RAY), "b%d.ray" % b)
    dsc.close()


def test_accumulate_equals_golden(rnd):
    g = gold("accumulate.npz")
    n = 32 * 16
    dh = torch.zeros((n, 4), dtype=torch.float32, device=rnd.device)
    dn = torch.zeros(n, dtype=torch.int32, device=rnd.device)
    f = 0
    while "in%d" % f in g:
        dc = torch.from_numpy(g["in%d" % f]).to(rnd.device)
        rnd.accumulate(dc, dh, dn, 8)
        assert_bits_equal(dc.cpu().numpy(), g["disp%d" % f], "display%d" % f)
        assert_bits_equal(dh.cpu().numpy(), g["hist%d" % f], "hist%d" % f)
        assert_bits_equal(dn.cpu().numpy(), g["count%d" % f], "count%d" % f)
        f += 1


IMAGES = [("c1_cbox", scenes.cbox, scenes.CBOX_CAM), ("mis64", scenes.mis, scenes.MIS_CAM),
          ("cboxdiff64", scenes.cbox_diffuse, scenes.CBOX_CAM)]


@pytest.mark.parametrize("name,getter,cam", IMAGES)
@pytest.mark.parametrize("mode", [L.MODE_EXACT, L.MODE_NOPRUNE])
def test_image_equals_golden(rnd, name, getter, cam, mode):
    """C1 (BASELINE configs[0]: cbox 256^2, 16 spp, depth 4) and two small
    images, whole frame loop, bit for bit against the reference kernels."""
    g = gold("image_%s.npz" % name)
    w, h, depth, frames, att = (int(x) for x in g["meta"])
    dsc = rnd.upload(getter())
    st = rnd.new_state(w, h, g["seeds_in"])
    rnd.render_frames(dsc, S.parse_camera(cam), st, depth, att, frames, mode=mode)
    torch.cuda.synchronize()
    assert_bits_equal(st.count.cpu().numpy(), g["count"], "count")
    assert_bits_equal(st.seeds_np(), g["seeds"], "seeds")
    assert_bits_equal(st.hist.cpu().numpy(), g["hist"], "hist")
    dsc.close()


def test_c1_hdr_dump_equals_stb_of_reference_image(rnd, tmp_path):
    """ColorOut's dump: our .hdr of our C1 image == the .hdr bytes of the
    reference image (writer pinned to stb in the CPU suite)."""
    g = gold("image_c1_cbox.npz")
    w, h, depth, frames, att = (int(x) for x in g["meta"])
    dsc = rnd.upload(scenes.cbox())
    st = rnd.new_state(w, h, g["seeds_in"])
    rnd.render_frames(dsc, S.parse_camera(scenes.CBOX_CAM), st, depth, att, frames)
    mine = S.encode_hdr(st.image())
    ref = S.encode_hdr(g["hist"].reshape(h, w, 4))
    assert mine == ref
    dsc.close()


def test_full_size_properties(rnd):
    """BASELINE configs[1] size (C2: 1024^2, depth 8, diffuse): deterministic,
    stripe partition (2 'GPUs', run in turn) bit-identical to 1, counts
    bounded by frames, radiance finite and non-negative."""
    data, cam = scenes.cbox_diffuse(), S.parse_camera(scenes.CBOX_CAM)
    w = h = 1024
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    outs = []
    for stripes in (1, 1, 2):
        st = rnd.new_state(w, h, seeds)
        for k in range(stripes):
            rnd.render_frames(dsc, cam, st, 8, 256, 3, stripe_rows=16, stripe_index=k, stripe_count=stripes)
        torch.cuda.synchronize()
        outs.append((st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()))
    for o in outs[1:]:
        for a, b, what in zip(outs[0], o, ("hist", "count", "seeds")):
            assert_bits_equal(a, b, what)
    hist, cnt, _ = outs[0]
    assert np.isfinite(hist).all() and (hist >= 0).all() and (hist[:, 3] == 0).all()
    assert cnt.min() >= 0 and cnt.max() <= 3
    assert (hist[cnt == 0] == 0).all()
    dsc.close()


def test_hip_vs_cpu_oracle_statistical(rnd):
    """HIP path vs the CPU restatement on the same seeded C1 input: the same
    envelope the oracle itself keeps against the reference (test_cpu.py)."""
    g = gold("image_c1_cbox.npz")
    w, h, depth, frames, att = (int(x) for x in g["meta"])
    st = rnd.new_state(w, h, g["seeds_in"])
    dsc = rnd.upload(scenes.cbox())
    rnd.render_frames(dsc, S.parse_camera(scenes.CBOX_CAM), st, depth, att, frames)
    mine = st.hist.cpu().numpy()
    px = np.arange(0, w * h, 4, dtype=np.int32)
    oh, oc, _, _ = O.render(scenes.cbox(), S.parse_camera(scenes.CBOX_CAM), w, h, depth, frames, att, g["seeds_in"],
                            pixels=px)
    close = (np.abs(mine[px] - oh[px]) <= 1e-5 * np.maximum(np.abs(oh[px]), 1e-3)).all(axis=1)
    assert close.mean() >= 0.97
    rel = np.abs(mine[px, :3].mean(0) - oh[px, :3].mean(0)) / oh[px, :3].mean(0)
    assert (rel < 0.01).all()
    dsc.close()


def test_kernel_stripes_follow_dist_owned_rows(rnd):
    """k_render's stripe mapping == dist.owned_rows: a rank touches exactly its
    pixels and produces there what the single-GPU render produces."""
    from montecarlopathtracing_amd import dist as D
    w, h, sr, world = 40, 41, 8, 3
    data, cam = scenes.cbox(), S.parse_camera(scenes.CBOX_CAM)
    seeds = R.default_seeds(w * h)
    dsc = rnd.upload(data)
    full = rnd.new_state(w, h, seeds)
    rnd.render_frames(dsc, cam, full, 4, 8, 3)
    for k in range(world):
        st = rnd.new_state(w, h, seeds)
        rnd.render_frames(dsc, cam, st, 4, 8, 3, stripe_rows=sr, stripe_index=k, stripe_count=world)
        m = D.ownership_mask(w, h, sr, k, world)
        hs, cs, ss = st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()
        assert (hs[~m] == 0).all() and (cs[~m] == 0).all() and np.array_equal(ss[~m], seeds[~m])
        assert hs[m].tobytes() == full.hist.cpu().numpy()[m].tobytes()
        assert np.array_equal(cs[m], full.count.cpu().numpy()[m])
        assert np.array_equal(ss[m], full.seeds_np()[m])
    dsc.close()


@pytest.mark.parametrize("variant", ["", "15"])
def test_app_from_config_json_reproduces_c1(tmp_path, variant):
    """The reference application loop driven by config.json (configid 2 = C1)
    reproduces the reference APPLICATION's image — the reference kernels over
    the GPU-treelet tree SceneCL renders over (scenebuild.cpp:87-95; golden
    image_c1_app.npz, tools/make_goldens.py app) — for splitmix seeds and for
    MSVC rand()'s 15-bit seeds (scenebuild.cpp:116-118, variant "15"), and
    dumps <objname>.hdr like ColorOut."""
    import hashlib

    from montecarlopathtracing_amd.app import App
    g = gold("image_c1_app.npz")
    app = App(scenes.CFG, configid=2, seeds=g["seeds_in" + variant], out_dir=str(tmp_path))
    app.init()
    assert hashlib.sha256(app.data.nodes.tobytes()).hexdigest() == str(g["nodes_sha256"])
    app.update(16)                      # frames 0..15 (attempt = 16: all accumulate)
    assert app.dumped is None           # dump happens after attempt + 1 frames
    assert_bits_equal(app.state.count.cpu().numpy(), g["count" + variant], "app count")
    assert_bits_equal(app.state.seeds_np(), g["seeds" + variant], "app seeds")
    assert_bits_equal(app.state.hist.cpu().numpy(), g["hist" + variant], "app hist")
    app.update(1)
    assert app.dumped and os.path.basename(app.dumped) == "cbox.obj.hdr"
    assert open(app.dumped, "rb").read() == S.encode_hdr(app.image())
    # ColorOut's display pass after the history is complete: frameBuffer, gamma 2.2
    pv = app.preview()
    ref = gamma_reference(app.image())
    assert_within_ulp(pv, ref, 1, "preview")


def gamma_reference(c):
    """testkernel.cl func in float64: pow(c, 1/2.2f) per channel (the float
    constant), rounded to float32; w = 0."""
    with np.errstate(invalid="ignore", over="ignore"):
        out = np.power(c.astype(np.float64), np.float64(np.float32(1) / np.float32(2.2))).astype(np.float32)
    out[..., 3] = 0.0
    return out


def assert_within_ulp(a, b, ulp, what):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    nan = np.isnan(b)
    assert np.array_equal(np.isnan(a), nan), what + ": NaN pattern"
    ia = a[~nan].view(np.int32).astype(np.int64)
    ib = b[~nan].view(np.int32).astype(np.int64)
    d = np.abs(ia - ib)
    assert np.all(np.sign(a[~nan]) == np.sign(b[~nan])) and d.max(initial=0) <= ulp, \
        "%s: %d values beyond %d ulp (max %d)" % (what, int((d > ulp).sum()), ulp, int(d.max(initial=0)))


def test_gamma_preview_is_opencl_pow(rnd):
    """testkernel.cl func: pow(c, 1/2.2f) per channel with OpenCL's pow (ocml;
    the reference kernel writes an RGBA32F image, and MI355X's runtime refuses
    image objects -- hipMallocArray(..., hipArraySurfaceLoadStore) returns
    "operation not supported" on the box (round 6) -- so it
    cannot run here; the bar is the correctly rounded value within 1 ulp
    plus exact special cases), w = 0, in place too."""
    rng = np.random.default_rng(7)
    vals = np.concatenate([
        rng.random(40000, dtype=np.float32),                       # the usual [0, 1) radiance
        rng.random(20000, dtype=np.float32) * np.float32(100.0),   # lights, over-exposed means
        np.float32(2.0) ** rng.integers(-149, 127, 4000).astype(np.float32),  # every binade, subnormals
        np.array([0.0, -0.0, 1.0, np.inf, np.nan, -1.0, -0.5, 1e-45, 3.4e38], np.float32),
    ]).astype(np.float32)
    vals = np.concatenate([vals, np.zeros((-len(vals)) % 4, np.float32)])
    col = vals.reshape(-1, 4)
    dev = torch.from_numpy(col.copy()).to(rnd.device)
    out = rnd.gamma_preview(dev).cpu().numpy()
    ref = gamma_reference(col)
    assert np.all(out[:, 3] == 0.0) and not np.signbit(out[:, 3]).any()
    assert_within_ulp(out[:, :3], ref[:, :3], 1, "gamma")
    sp = out[:, :3].ravel()[np.isin(col[:, :3].ravel(), [0.0, 1.0, np.inf])]
    assert np.array_equal(sp, np.power(col[:, :3].ravel()[np.isin(col[:, :3].ravel(), [0.0, 1.0, np.inf])], 1.0))
    rnd.gamma_preview(dev, out=dev)                                # in place
    assert np.array_equal(dev.cpu().numpy().view(np.int32), out.view(np.int32))
    for bad in (torch.empty(dev.numel() - 4, device=rnd.device),   # too small
                torch.empty(dev.shape[::-1], device=rnd.device).t(),  # strided
                torch.empty(dev.shape, dtype=torch.float64, device=rnd.device),
                torch.empty(dev.shape)):                           # host
        with pytest.raises(L.MCPTError):
            rnd.gamma_preview(dev, out=bad)


def test_cli_runs(tmp_path):
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-m", "montecarlopathtracing_amd", scenes.CFG, "--configid", "2",
                        "--out", str(tmp_path), "--frames", "2", "--preview", str(tmp_path / "cbox.png")],
                       cwd=scenes.ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(tmp_path / "cbox.obj.hdr")
    PIL = pytest.importorskip("PIL.Image")
    with PIL.open(tmp_path / "cbox.png") as im:
        assert im.size == (256, 256) and im.mode == "RGB"


def _build_cases():
    rng = np.random.default_rng(7)
    tri = rng.uniform(-3, 3, (50, 3, 3)).astype(np.float32)
    dup = np.concatenate([np.repeat(tri[:1], 300, axis=0), tri])  # equal Morton codes: middle splits
    flat = tri.copy()
    flat[:, :, 2] = 0.0  # a flat axis: 0/0 in the code -> 0
    cases = {"one": tri[:1], "two": tri[:2], "three": tri[:3], "dup": dup, "flat": flat,
             "signed_zero": np.where(np.abs(tri) < 0.5, np.float32(-0.0), tri).astype(np.float32)}
    return cases


@pytest.mark.parametrize("name", ["cbox", "mis", "random200k", "one", "two", "three", "dup", "flat", "signed_zero"])
def test_gpu_hlbvh_build_equals_host(name):
    """the reference HLBVH built on the GPU is the host
    build (hlbvh.cpp restated in mcpt_host.cpp, pinned to the C oracle) bit for bit."""
    if name == "cbox":
        tris = scenes.cbox().tris
    elif name == "mis":
        tris = scenes.mis().tris
    elif name == "random200k":
        tris = S.random_mesh(200_000).tris
    else:
        v = _build_cases()[name]
        t = np.zeros(len(v), L.TRIANGLE)
        t["v"][:, :, :3] = v
        tris = S.pack_triangles(t, np.zeros(len(v), np.int32))
    host = S.build_hlbvh(tris)
    dev = R.records(R.build_hlbvh_device(tris), L.BVHNODE)
    assert_bits_equal(dev, host, "hlbvh nodes")
