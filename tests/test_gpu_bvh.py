"""GPU BVH passes against their CPU restatements.

TreeletBVH<GPU> (MCPT/kernels/treeletBVH.cl, the pass every reference render
runs, scenebuild.cpp:87-95) is mcpt_treelet_gpu_device; its oracle is the
sequential restatement oracle/mcpt_oracle_treelet_gpu.cpp (parity unpinned:
the reference kernel does not compile).

TreeletBVH<CPU> (MCPT/BVH/treeletBVH.cpp, "bvhtype": "treelet") runs on the
GPU as mcpt_treelet_device; the oracle (oracle/mcpt_oracle_treelet.cpp) is the
reference's sequential pass written with the same std::push_heap/pop_heap
calls.  Bar: node arrays bit-identical.  The oracle is itself pinned by the
reference's own TreeletBVH<CPU>, compiled unmodified (oracle/ref_host_golden,
tests/golden/ref_host.npz), and the GPU pass is compared with those fixtures
directly below.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import bvhtest as B  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402

from . import oracle as O  # noqa: E402
from . import scenes  # noqa: E402
from .test_gpu_golden import _build_cases  # noqa: E402
from .test_gpu_parity import assert_bits_equal  # noqa: E402


def _tris(v):
    t = np.zeros(len(v), L.TRIANGLE)
    t["v"][:, :, :3] = v
    return S.pack_triangles(t, np.zeros(len(v), np.int32))


def _case(name):
    if name == "cbox":
        return scenes.cbox().tris
    if name == "mis":
        return scenes.mis().tris
    if name == "random200k":
        return S.random_mesh(200_000).tris
    if name.startswith("rand"):
        n = int(name[4:])
        rng = np.random.default_rng(n)
        return _tris(rng.uniform(-2, 2, (n, 3, 3)).astype(np.float32))
    return _tris(_build_cases()[name])


CASES = ["cbox", "mis", "random200k", "two", "three", "dup", "flat", "signed_zero"] + \
        ["rand%d" % k for k in (4, 5, 6, 7, 8, 9, 13, 64, 1000)]


@pytest.mark.parametrize("name", CASES)
def test_gpu_treelet_equals_oracle(name):
    tris = _case(name)
    nodes = S.build_hlbvh(tris)
    rc, ref = O.treelet(nodes)
    if rc == -1:
        with pytest.raises(L.MCPTError):
            R.treelet_device(nodes)
        return
    assert rc == 0
    mine = R.treelet_device(nodes)
    assert_bits_equal(mine, ref, "treelet nodes")


def test_gpu_treelet_on_device_built_hlbvh():
    """The GPU pipeline end to end: HLBVH built on the GPU, then treelets, in
    HBM, equals the oracle's pass over the host build."""
    tris = S.random_mesh(100_000, seed=5).tris
    d = R.build_hlbvh_device(tris)
    R.treelet_device(d)
    _, ref = O.treelet(S.build_hlbvh(tris))
    assert_bits_equal(R.records(d, L.BVHNODE), ref, "device pipeline")


def test_gpu_treelet_recursion_cycle_is_an_error():
    n = 40
    x = np.arange(n, dtype=np.float32)
    v = np.zeros((n, 3, 3), np.float32)
    v[:, 0, 0], v[:, 1, 0], v[:, 2, 0] = x, x + 0.5, x
    v[:, 2, 1] = 0.5
    nodes = S.build_hlbvh(_tris(v))
    assert O.treelet(nodes)[0] == -1
    with pytest.raises(L.MCPTError, match="does not terminate"):
        R.treelet_device(nodes)


# ------------------------------------ TreeletBVH<GPU> (treeletBVH.cl)
def _gpu_rcp_bits(nodes):
    """v_rcp_f32 of frexp_mant(rootArea) on this GPU, the one hardware value
    the CPU restatement of treeletBVH.cl's 2.5-ulp division takes as input."""
    from . import refgpu
    if not refgpu.available():
        pytest.skip("oracle/_ref not built")
    return int(refgpu.rcp_f32(O.root_area_mant(nodes))[0].view(np.uint32))


def _treelet_gpu_ref(nodes):
    rc, out, st = O.treelet_gpu(nodes, rcp_bits=_gpu_rcp_bits(nodes))
    assert rc == 0
    return out, st


@pytest.mark.parametrize("name", CASES + ["dining"])
def test_gpu_treelet_gpu_equals_oracle(name):
    """mcpt_treelet_gpu_device (csrc/mcpt_treelet_gpu.hip: one launch per depth,
    one wave per node) == the sequential leaf-walk restatement of
    treeletBVH.cl (oracle/mcpt_oracle_treelet_gpu.cpp), node arrays bit for bit."""
    tris = scenes.dining().tris if name == "dining" else _case(name)
    nodes = S.build_hlbvh(tris)
    ref, st = _treelet_gpu_ref(nodes)
    mine = R.treelet_gpu_device(nodes)
    assert_bits_equal(mine, ref, "treelet_gpu nodes")
    _, cpu = O.treelet(nodes)
    if len(tris) >= 64:  # the CPU pass (heap queue, /rootArea refit) builds another tree
        assert cpu.tobytes() != mine.tobytes()


def test_gpu_treelet_gpu_on_device_built_hlbvh_1m():
    """HLBVH built on the GPU then the GPU treelet pass, in HBM, on a
    1M-triangle random mesh (C5's kind of scene): equals the oracle's pass
    over the host build."""
    tris = S.random_mesh(1_000_000, seed=7).tris
    d = R.build_hlbvh_device(tris)
    R.treelet_gpu_device(d)
    host = S.build_hlbvh(tris)
    ref, st = _treelet_gpu_ref(host)
    assert_bits_equal(R.records(d, L.BVHNODE), ref, "device pipeline")
    assert st[6] == 0


def test_gpu_treelet_gpu_c5_10m():
    """C5's own tree at full size: the 10 M-triangle
    random mesh (seed 42, +2 light triangles) built as bench.py --workload C5
    builds it -- the GPU HLBVH, then the GPU treelet pass, in HBM -- equals
    the oracle's sequential treelet pass over the host HLBVH, node for node."""
    tris = S.random_mesh(10_000_000, build=lambda t: None).tris
    d = R.build_hlbvh_device(tris)
    R.treelet_gpu_device(d)
    mine = R.records(d, L.BVHNODE)
    del d
    host = S.build_hlbvh(tris)
    ref, st = _treelet_gpu_ref(host)
    del host
    assert len(mine) == 2 * len(tris) - 1
    assert_bits_equal(mine, ref, "C5 device pipeline")
    assert st[6] == 0


def test_gpu_treelet_gpu_rejects_non_hlbvh_layout():
    nodes = S.build_hlbvh(_case("rand64"))
    bad = nodes.copy()
    bad[3]["left"] = bad[3]["right"]  # an internal slot that reads as a leaf
    with pytest.raises(L.MCPTError, match="HLBVH layout"):
        R.treelet_gpu_device(bad)
    with pytest.raises(L.MCPTError, match="2n-1"):
        R.treelet_gpu_device(nodes[:-1])


@pytest.mark.parametrize("bvhtype", ["hlbvh", "treelet", "treeletGPU"])
def test_app_renders_over_the_gpu_treelet_tree_for_every_bvhtype(tmp_path, bvhtype):
    """SceneCL's ctor falls through into its GPUBVH block for every bvhtype
    (scenebuild.cpp:66-95): the App uploads exactly the GPU treelet tree of a
    fresh HLBVH, whatever the config names, and renders over it."""
    import json

    from montecarlopathtracing_amd import config as C
    from montecarlopathtracing_amd.app import App
    obj = C.Config(scenes.CFG, configid=2).root
    obj = json.loads(json.dumps(obj))
    obj["config"][2]["bvhtype"] = bvhtype
    obj["config"][2]["width"] = obj["config"][2]["height"] = 32
    obj["config"][2]["camera"]["resolution"] = [32, 32]
    obj["config"][2]["directory"] = scenes.ROOT + "/scenes/cbox/"
    app = App(C.Config(obj, configid=2), out_dir=str(tmp_path), root="/")
    app.init()
    ref, _ = _treelet_gpu_ref(scenes.cbox().nodes)
    assert_bits_equal(app.data.nodes, ref, "app nodes")
    app.update(2)
    assert app.state.count.cpu().numpy().sum() > 0


def test_app_unknown_bvhtype_raises():
    from montecarlopathtracing_amd import config as C
    from montecarlopathtracing_amd.app import App
    obj = dict(C.Config(scenes.CFG, configid=2).root)
    obj["config"] = [dict(c) for c in obj["config"]]
    obj["config"][2]["bvhtype"] = "sah"
    app = App(C.Config(obj, configid=2), root=scenes.ROOT)
    with pytest.raises(ValueError, match="BVH Not Implemented"):
        app.init()


# ------------------------------------------------------ testbvh metrics
from . import refgpu  # noqa: E402

needs_ref = pytest.mark.skipif(not refgpu.available(), reason="oracle/_ref not built")

METRIC_SCENES = [("cbox", "scenes/cbox/", "cbox.obj", scenes.CBOX_CAM), ("mis", "scenes/veach_mis/", "mis.obj",
                                                                         scenes.MIS_CAM)]


def _metric_tris(d, obj):
    return B.load_triangles(scenes.ROOT + "/" + d, obj)


@needs_ref
@pytest.mark.parametrize("bvhtype", ["hlbvh", "treelet", "treeletGPU"])
@pytest.mark.parametrize("name,d,obj,cam", METRIC_SCENES)
def test_epo_per_triangle_bitexact_vs_reference_kernel(name, d, obj, cam, bvhtype):
    """EPO_GPU: mcpt_bvh_epo_device's per-triangle EPO and area equal the
    reference's EPO.cl kernel (compiled unmodified for gfx950) bit for bit."""
    tris = _metric_tris(d, obj)
    nodes = B.build(tris, bvhtype)
    val, e, a, ovf = B.epo(nodes, tris, per_triangle=True)
    re, ra = refgpu.epo(nodes, tris)
    assert_bits_equal(a, ra, "triangle area")
    if ovf == 0:
        assert_bits_equal(e, re, "epo")
    else:  # the reference overflows its points[8] there (undefined behaviour)
        assert (e == re).mean() > 0.999
    ref_val = np.float32(np.sum(re, dtype=np.float64) / np.sum(ra, dtype=np.float64))
    assert np.float32(val) == ref_val


def test_epo_random_mesh_bitexact_vs_reference_kernel():
    if not refgpu.available():
        pytest.skip("oracle/_ref not built")
    tris = S.random_mesh(20_000, seed=11).tris
    nodes = S.build_hlbvh(tris)
    _, e, a, ovf = B.epo(nodes, tris, per_triangle=True)
    re, ra = refgpu.epo(nodes, tris)
    assert_bits_equal(a, ra, "triangle area")
    assert ovf == 0
    assert_bits_equal(e, re, "epo")


@pytest.mark.parametrize("bvhtype", ["hlbvh", "treelet", "treeletGPU"])
@pytest.mark.parametrize("name,d,obj,cam", METRIC_SCENES)
def test_lcv_counts_equal_oracle(name, d, obj, cam, bvhtype):
    """LCV: per-ray leaf counts on the GPU equal the CPU restatement of
    bvhtest.cpp:324-444 exactly (host float semantics on both sides)."""
    tris = _metric_tris(d, obj)
    nodes = B.build(tris, bvhtype)
    camera = S.parse_camera(cam)
    w, h = 160, 120
    v, counts = B.lcv(nodes, camera, w, h, counts=True)
    ov, ocounts = O.bvh_lcv(nodes, camera, w, h)
    assert (counts == ocounts).all()
    assert np.float32(v) == np.float32(ov)


@pytest.mark.parametrize("bvhtype", ["hlbvh", "treelet", "treeletGPU"])
def test_sah_equals_oracle(bvhtype):
    tris = _metric_tris("scenes/cbox/", "cbox.obj")
    nodes = B.build(tris, bvhtype)
    assert np.float32(B.sah(nodes)) == np.float32(O.bvh_sah(nodes))


def test_cli_testbvh_and_testall():
    """main.cpp:14-19 mode dispatch: config 5 (testbvh, treelet, camera) and
    config 6 (testall) print the reference's metric lines."""
    import subprocess
    import sys
    for cid, want in ((5, ("cbox.obj 33490", "treelet", "SAH: ", "EPO_GPU: ", "LCV: ")),
                      (6, ("mis.obj 3812", "hlbvh", "SAH: ", "EPO_GPU: "))):
        r = subprocess.run([sys.executable, "-m", "montecarlopathtracing_amd", scenes.CFG, "--configid", str(cid)],
                           cwd=scenes.ROOT, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        for w in want:
            assert w in r.stdout, r.stdout


# ------------------------------------------- the reference's own host C++
def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["cbox", "mis", "random20k"])
def test_gpu_treelet_equals_reference_host(name):
    """mcpt_treelet_device == TreeletBVH<CPU> (BVH/treeletBVH.cpp:30-372)
    compiled unmodified from the reference (tests/golden/ref_host.npz,
    tools/make_host_goldens.py), byte for byte."""
    g = np.load(os.path.join(scenes.ROOT, "tests", "golden", "ref_host.npz"))
    nodes = {"cbox": lambda: scenes.cbox().nodes, "mis": lambda: scenes.mis().nodes,
             "random20k": lambda: S.random_mesh(20_000, seed=11).nodes}[name]()
    assert _sha(nodes) == str(g["treelet_%s_in_sha" % name])
    assert _sha(R.treelet_device(nodes)) == str(g["treelet_%s_out_sha" % name])


def test_gpu_lcv_equals_reference_host():
    """mcpt_bvh_lcv_device == BVH::TEST::LCV (bvhtest.cpp:324-444) compiled
    from the reference (cbox, config 2's 256 x 256), float bits."""
    g = np.load(os.path.join(scenes.ROOT, "tests", "golden", "ref_host.npz"))
    w, h = (int(x) for x in g["lcv_size"])
    v = B.lcv(scenes.cbox().nodes, S.parse_camera(scenes.CBOX_CAM), w, h)
    assert np.float32(v).view(np.uint32) == g["lcv_cbox_bits"]


# ------------------------------------ the scene's structures built on the GPU
UPLOAD_CASES = ["cbox", "mis", "dining", "two", "three", "dup", "flat", "signed_zero", "rand5", "rand64", "rand1000",
                "random200k"]


class _Scene:  # what DeviceScene reads of a SceneData
    def __init__(self, tris, nodes, mats):
        self.tris, self.nodes, self.mats = tris, nodes, mats


def _upload_both(tris, nodes, mats):
    rnd = R.Renderer(0)
    host = rnd.upload(_Scene(tris, nodes, mats))
    dev = rnd.upload((R.to_device(tris, 0), R.to_device(nodes, 0), mats))
    return rnd, host, dev


@pytest.mark.parametrize("name", UPLOAD_CASES)
def test_scene_upload_device_equals_host(name):
    """mcpt_scene_upload_device (csrc/mcpt_upload.hip: validation, stack
    bounds, the reference tree 4-wide, the binned-SAH search tree with its
    4-wide collapse and emission order, the quantized nodes, the triangle
    records, all on the GPU) == mcpt_scene_upload (host, mcpt_sah.cpp): every
    device array byte for byte."""
    named = {"cbox": scenes.cbox, "mis": scenes.mis, "dining": scenes.dining}
    if name in named:
        d = named[name]()
        tris, mats = d.tris, d.mats
    else:
        tris, mats = _case(name), scenes.cbox().mats
    nodes = R.treelet_gpu_device(S.build_hlbvh(tris))
    rnd, host, dev = _upload_both(tris, nodes, mats)
    for k in R.DeviceScene.ARRAYS + ("meta",):
        a, b = host.read(k), dev.read(k)
        assert a.tobytes() == b.tobytes(), (name, k, len(a), len(b))
    host.close()
    dev.close()
    rnd.close()


def test_scene_upload_device_c5_size_renders_bitexact():
    """A 2M-triangle random mesh (C5's kind, large ranges split level by level
    on the GPU): the device-built scene equals the host-built one array for
    array, and renders the same bits."""
    tris = S.random_mesh(2_000_000, seed=3, build=lambda t: None).tris
    d = R.build_hlbvh_device(tris)
    R.treelet_gpu_device(d)
    nodes = R.records(d, L.BVHNODE).copy()
    mats = S.random_mesh(8, seed=3).mats
    rnd, host, dev = _upload_both(tris, nodes, mats)
    for k in R.DeviceScene.ARRAYS + ("meta",):
        assert host.read(k).tobytes() == dev.read(k).tobytes(), k
    cam = S.parse_camera(S.RANDOM_MESH_CAMERA)
    out = []
    for sc in (host, dev):
        st = rnd.new_state(96, 64)
        rnd.render_frames(sc, cam, st, 4, 8, 3)
        out.append((st.hist.cpu().numpy(), st.seeds_np()))
    assert out[0][0].tobytes() == out[1][0].tobytes() and np.array_equal(out[0][1], out[1][1])
    host.close()
    dev.close()
    rnd.close()
