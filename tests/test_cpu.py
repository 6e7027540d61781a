"""CPU suite (no GPU): the boundary library, the host pipeline and the CPU
oracle, pinned against the reference's own outputs in tests/golden/.

Golden provenance (tools/make_goldens.py):
  rays/chain_*/accumulate/image_*.npz — the reference's OpenCL kernels compiled
      unmodified for gfx950 and run on an MI355X (tests/refgpu.py);
  tinyobj_*.npz, stb_*.hdr — the reference's vendored tinyobjloader and
      stb_image_write compiled from /root/reference (oracle/_ref/libref_io.so).
"""
import ctypes
import json
import os
import sys
import re

import numpy as np
import pytest

from montecarlopathtracing_amd import _lib as L
from montecarlopathtracing_amd import config as C
from montecarlopathtracing_amd import render as R
from montecarlopathtracing_amd import scene as S

from . import oracle as O
from . import scenes

ROOT = scenes.ROOT
GOLD = os.path.join(ROOT, "tests", "golden")


def gold(name):
    return np.load(os.path.join(GOLD, name))


# ------------------------------------------------------------------ boundary
def test_abi_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "mcpt_hip.h")).read()
    declared = set(re.findall(r"\b(mcpt_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(L.SIGNATURES), declared ^ set(L.SIGNATURES)
    so = ctypes.CDLL(L.LIB_PATH)
    for name in declared:
        assert hasattr(so, name), name
    assert L.lib().mcpt_version().decode().startswith("mcpt-mi355x")


def _header_fields(hdr, struct):
    """int32 field names of `typedef struct <struct> {...}` in header order."""
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), hdr, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";"):
        m = re.match(r"\s*int32_t\s+(.*)", decl, re.S)
        if m:
            names += [n.strip() for n in m.group(1).split(",")]
    return names


def test_tuning_and_params_structs_match_header():
    """mcpt_tuning grows at its end as knobs are added: the ctypes mirrors
    (_lib.Tuning, _lib.RenderParams) must list the header's int32 fields in its
    order, or Python would set the wrong knob."""
    hdr = open(os.path.join(ROOT, "include", "mcpt_hip.h")).read()
    assert [f for f, _ in L.Tuning._fields_] == _header_fields(hdr, "mcpt_tuning")
    assert [f for f, _ in L.RenderParams._fields_] == _header_fields(hdr, "mcpt_render_params")


def test_abi_struct_sizes_match_header(tmp_path):
    """The ctypes mirrors of every struct that crosses the ABI have the C
    compiler's size for the header's definition (mcpt_stats grows at its end
    too), and the library reports the header's ABI revision."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "mcpt_hip.h"\nint main(void) { printf("%zu %zu %zu %d\\n", '
                   'sizeof(mcpt_stats), sizeof(mcpt_tuning), sizeof(mcpt_render_params), MCPT_ABI_VERSION); '
                   'return 0; }\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    st, tu, rp, abi = (int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                                      check=True).stdout.split())
    assert (st, tu, rp) == (ctypes.sizeof(L.Stats), ctypes.sizeof(L.Tuning), ctypes.sizeof(L.RenderParams))
    assert abi == L.ABI_VERSION == L.lib().mcpt_abi_version()


def test_record_layouts_match_objdef():
    # objdef.h:21-99 sizes; the C structs are checked by the same numbers in the ABI tests below
    assert (L.CAMERA.itemsize, L.RAY.itemsize, L.HIT.itemsize) == (80, 48, 48)
    assert (L.TRIANGLE.itemsize, L.MATERIAL.itemsize, L.BVHNODE.itemsize) == (64, 48, 64)
    assert L.HIT.fields["t"][1] == 32 and L.HIT.fields["material_id"][1] == 40
    assert L.BVHNODE.fields["left"][1] == 52 and L.CAMERA.fields["arg"][1] == 64


def test_abi_errors_are_status_codes():
    lib = L.lib()
    nodes = np.zeros(1, L.BVHNODE)
    assert lib.mcpt_build_hlbvh(None, 0, L.ptr(nodes)) == -1
    assert b"empty" in lib.mcpt_last_error()
    nt, nm = ctypes.c_int64(0), ctypes.c_int32(0)
    assert lib.mcpt_load_obj(b"/nonexistent/", b"x.obj", None, None, ctypes.byref(nt), None, ctypes.byref(nm)) == -3
    img = np.zeros((4, 4, 4), np.float32)
    assert lib.mcpt_write_hdr(b"/nonexistent/dir/x.hdr", 4, 4, L.ptr(img), 1) == -3
    with pytest.raises(L.MCPTError):
        L.check(lib.mcpt_build_hlbvh(None, 0, None))
    with pytest.raises(ValueError):
        S.build_hlbvh(np.zeros(0, L.TRIANGLE))


def test_product_has_no_cpu_fallback(monkeypatch):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(L.MCPTError):
        R.Renderer(0)


# -------------------------------------------------------------------- config
def test_config_hash_comments_and_getters():
    text = '{ "config": [ { "width": 512.7, "height": 256, # comment "x"\n "directory": "a#b/", "objname": "o.obj",' \
           ' "maxdepth": 4, "attempt": 8, "opencl": true, "platform": "p", "camera": {"fov": 1} } ], # tail\n' \
           ' "configid": 0 }'
    c = C.Config(C.loads(text))
    assert c.WIDTH() == 512 and c.HEIGHT() == 256 and c.GETDIRECTORY() == "a#b/"
    assert c.MAXDEPTH() == 4 and c.MAXATTEPMT() == 8 and c.BVHTYPE() == "hlbvh" and c.USEOPENCL()


def test_repo_config_json_parses():
    root = C.loads(open(scenes.CFG).read())
    for i in range(len(root["config"])):
        c = C.Config(root, i)
        assert os.path.exists(os.path.join(ROOT, c.GETDIRECTORY(), c.GETOBJNAME()))
    assert C.Config(scenes.CFG).MAXDEPTH() == 4  # configid 2 = C1


# ------------------------------------------------------------ scene loading
@pytest.mark.parametrize("d,obj", [("cbox", "cbox.obj"), ("veach_mis", "mis.obj"), ("diningroom", "diningroom.obj")])
def test_obj_loader_matches_reference_tinyobj(d, obj):
    g = gold("tinyobj_%s.npz" % d)
    tris, mats, idx = S.load_object(os.path.join(ROOT, "scenes", d) + "/", obj)
    v = np.ascontiguousarray(tris["v"][:, :, :3].reshape(-1, 9))
    assert np.array_equal(v.view(np.uint32), g["verts"].view(np.uint32))
    assert np.array_equal(idx, g["matids"])
    # materials: the reference classification of tinyobj's raw records
    for m, raw in zip(mats, g["mtl"]):
        ref = S.classify_material(raw[0], raw[1:4], raw[4:7], raw[7:10], raw[10])
        assert m.tobytes() == ref.tobytes()
    meta = json.load(open(os.path.join(GOLD, "cpu_fixtures.json")))[d]
    assert len(tris) == meta["triangles"] and len(mats) == meta["materials"]


def test_material_classification_rules():
    # thirdpartywrapper.cpp:65-97 precedence and scaling, restated in numpy double
    pi = 3.14159265358
    m = S.classify_material(1.5, (5, 5, 5), (1, 1, 1), (1, 1, 1), 10)
    assert m["type"] == L.MCPT_TRANSPARENT and m["Ni"] == np.float32(1.5)
    m = S.classify_material(1.0, (0, 0.5, 0), (1, 1, 1), (1, 1, 1), 10)
    assert m["type"] == L.MCPT_LIGHT and list(m["ka_ks"]) == [0, 0.5, 0, 0]
    m = S.classify_material(1.0, (0, 0, 0), (0.25, 0.5, 0.75), (0.97, 0.99, 0.93), 98)
    assert m["type"] == L.MCPT_GLOSSY and m["Ns"] == 98
    ks = (np.float64(np.float32(98) + 2) * (2.0 / pi) * np.array([0.97, 0.99, 0.93], np.float32).astype(np.float64))
    assert np.array_equal(m["ka_ks"][:3], ks.astype(np.float32))
    kd = ((1.0 / pi) * np.array([0.25, 0.5, 0.75], np.float32).astype(np.float64)).astype(np.float32)
    assert np.array_equal(m["kd"][:3], kd)
    m = S.classify_material(1.0, (0, 0, 0), (0.25, 0.5, 0.75), (1, 1, 1), 1.0)
    assert m["type"] == L.MCPT_DIFFUSE and np.array_equal(m["kd"][:3], kd)


def test_pack_and_camera_match_oracle():
    tris, mats, idx = S.load_object(os.path.join(ROOT, "scenes/cbox/"), "cbox.obj")
    assert S.pack_triangles(tris, idx).tobytes() == O.pack_triangles(tris, idx).tobytes()
    for cj in (scenes.CBOX_CAM, scenes.MIS_CAM, scenes.DINING_CAM):
        assert S.parse_camera(cj).tobytes() == O.parse_camera(cj).tobytes()
    c = S.parse_camera(scenes.CBOX_CAM)[0]
    assert c["horizontal"][0] == -1.0  # cbox: image-left is +x (red wall), SURVEY §8(a)
    assert c["arg"] == np.float32(39.3077 * 3.14159265358 / 180.0)


# -------------------------------------------------------------------- HLBVH
def _rand_tris(n, seed, flat=False, dup=False):
    rng = np.random.default_rng(seed)
    c = rng.uniform(0, 100, (n, 3)).astype(np.float32)
    if dup:
        c[: n // 2] = c[0]
    v = c[:, None, :] + rng.uniform(-1, 1, (n, 3, 3)).astype(np.float32)
    if flat:
        v[:, :, 2] = 5.0
    t = np.zeros(n, L.TRIANGLE)
    t["v"][:, :, :3] = v
    return t


def _check_tree(nodes, n):
    assert len(nodes) == 2 * n - 1 and nodes[0]["parent"] == -1
    if n == 1:
        return
    leaves = sorted(int(nodes[i]["left"]) for i in range(n - 1, 2 * n - 1))
    assert leaves == list(range(n))
    for i in range(n - 1):
        l, r = int(nodes[i]["left"]), int(nodes[i]["right"])
        assert l != r and nodes[l]["parent"] == i and nodes[r]["parent"] == i
        for ch in (l, r):
            assert (nodes[i]["bbmin"] <= nodes[ch]["bbmin"]).all() and (nodes[i]["bbmax"] >= nodes[ch]["bbmax"]).all()


@pytest.mark.parametrize("case", ["cbox", "mis", "n1", "n2", "n3", "rand", "flat", "dup"])
def test_hlbvh_product_equals_oracle(case):
    if case in ("cbox", "mis"):
        t = (scenes.cbox() if case == "cbox" else scenes.mis()).tris
    else:
        n = {"n1": 1, "n2": 2, "n3": 3, "rand": 5000, "flat": 700, "dup": 900}[case]
        t = _rand_tris(n, 11, flat=(case == "flat"), dup=(case == "dup"))
    mine = S.build_hlbvh(t)
    ref = O.build_hlbvh(t)
    assert mine.tobytes() == ref.tobytes()
    _check_tree(mine, len(t))
    assert S.bvh_stack_depth(mine) <= 64


# --------------------------------------------------------------------- RGBE
@pytest.mark.parametrize("name", ["synthetic", "narrow"])
def test_rgbe_writer_matches_reference_stb(name, tmp_path):
    im = np.load(os.path.join(GOLD, "stb_%s_input.npy" % name))
    ref = open(os.path.join(GOLD, "stb_%s.hdr" % name), "rb").read()
    assert S.encode_hdr(im) == ref
    assert O.encode_hdr(im) == ref
    p = str(tmp_path / "x.hdr")
    S.write_hdr(p, im)
    assert open(p, "rb").read() == ref


def test_rgbe_edge_cases_product_equals_oracle():
    rng = np.random.default_rng(5)
    for w, h in ((1, 1), (7, 3), (8, 2), (300, 2), (129, 1)):
        im = rng.exponential(1.0, (h, w, 4)).astype(np.float32)
        im[..., :3][rng.random((h, w, 3)) < 0.3] = 0.0
        for flip in (0, 1):
            assert S.encode_hdr(im, flip) == O.encode_hdr(im, flip)


# ------------------------------------------- CPU oracle vs reference goldens
def _ulp(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)


CAMS = {"cbox": scenes.CBOX_CAM, "mis": scenes.MIS_CAM, "dining": scenes.DINING_CAM}


@pytest.mark.parametrize("k", list(CAMS))
def test_oracle_rays_vs_reference(k):
    """Tolerance: origins/ids exact; unit directions within 4e-7 absolute
    (the GPU normalises with the hardware rsq, the oracle with 1/sqrt)."""
    ref = gold("rays.npz")[k].view(L.RAY)
    mine = O.generate(S.parse_camera(CAMS[k]), 64, 48)
    assert mine["origin"].tobytes() == ref["origin"].tobytes()
    assert np.array_equal(mine["direction"][:, 3].view(np.int32), ref["direction"][:, 3].view(np.int32))
    assert np.abs(mine["direction"][:, :3] - ref["direction"][:, :3]).max() <= 4e-7


@pytest.mark.parametrize("name", ["cbox", "mis"])
def test_oracle_bounce_chain_vs_reference(name):
    """Per bounce, same inputs as the reference kernels got.  Discrete outputs
    exact (hit triangle/material, RNG seeds, terminate flags); t within 4 ulp
    for 99 % of hits; new directions within 2e-6; colours within 5e-3
    relative (glossy pow(cos, 4000) amplifies the 1-ulp built-in differences)."""
    c = gold("chain_%s.npz" % name)
    data = scenes.cbox() if name == "cbox" else scenes.mis()
    depth = int(c["depth"])
    for b in range(depth):
        rays = c["rays%d" % b].view(L.RAY)
        href = c["hits%d" % b].view(L.HIT)
        live = (rays["origin"][:, 3].view(np.int32) & np.int32(-16777216)) == 0
        h = O.intersect(data, rays, hits=c["hits_in%d" % b].view(L.HIT))
        assert np.array_equal(h["material_id"][live], href["material_id"][live])
        assert np.array_equal(h["triangle_id"][live], href["triangle_id"][live])
        hit = live & (href["t"] < 3e38)
        if hit.any():
            assert np.percentile(_ulp(h["t"][hit], href["t"][hit]), 99) <= 4
        r2, c2, s2 = O.shade(data, rays, href, c["colors_in%d" % b], c["seeds_in%d" % b], depth)
        rr = c["rays_out%d" % b].view(L.RAY)
        assert np.array_equal(s2, c["seeds%d" % b])
        assert np.array_equal(r2["origin"][:, 3].view(np.int32), rr["origin"][:, 3].view(np.int32))
        assert np.abs(r2["direction"][:, :3] - rr["direction"][:, :3]).max() <= 2e-6
        cref = c["colors%d" % b]
        assert (np.abs(c2 - cref) <= 5e-3 * np.maximum(np.abs(cref), 1e-6)).all()


def test_oracle_accumulate_vs_reference():
    g = gold("accumulate.npz")
    w, h = 32, 16
    hist = np.zeros((w * h, 4), np.float32)
    cnt = np.zeros(w * h, np.int32)
    f = 0
    while "in%d" % f in g:
        d, hist, cnt = O.accumulate(g["in%d" % f], hist, cnt, 8)
        assert np.array_equal(cnt, g["count%d" % f])
        assert np.abs(hist - g["hist%d" % f]).max() <= 2e-7 * max(1.0, float(np.abs(g["hist%d" % f]).max()))
        hist = g["hist%d" % f].copy()  # continue from the reference state
        f += 1
    assert f >= 8


@pytest.mark.parametrize("name,getter,cam,stride", [("c1_cbox", scenes.cbox, scenes.CBOX_CAM, 4),
                                                     ("mis64", scenes.mis, scenes.MIS_CAM, 1),
                                                     ("cboxdiff64", scenes.cbox_diffuse, scenes.CBOX_CAM, 1)])
def test_oracle_image_vs_reference(name, getter, cam, stride):
    """Whole-image parity of the CPU restatement against the reference kernels
    (same seeds).  Chaotic paths decorrelate after a 1-ulp built-in difference,
    so the bar is statistical, calibrated on the oracle's ulp envelope:
    >= 97 % of pixels within 1e-5 relative, >= 97 % identical sample counts,
    per-channel image mean within 1 %."""
    g = gold("image_%s.npz" % name)
    w, h, depth, frames, att = (int(x) for x in g["meta"])
    px = np.arange(0, w * h, stride, dtype=np.int32)
    hist, cnt, sd, _ = O.render(getter(), S.parse_camera(cam), w, h, depth, frames, att, g["seeds_in"], pixels=px)
    rh, mh = g["hist"][px], hist[px]
    close = (np.abs(mh - rh) <= 1e-5 * np.maximum(np.abs(rh), 1e-3)).all(axis=1)
    assert close.mean() >= 0.97, close.mean()
    assert (cnt[px] == g["count"][px]).mean() >= 0.97
    rel = np.abs(mh[:, :3].mean(0) - rh[:, :3].mean(0)) / rh[:, :3].mean(0)
    assert (rel < 0.01).all(), rel


@pytest.fixture(scope="module")
def sah_check_exe(tmp_path_factory):
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "montecarlopathtracing_amd", "csrc")
    exe = str(tmp_path_factory.mktemp("sah") / "sah_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", csrc, os.path.join(root, "tests", "native", "sah_check.cpp"),
                    os.path.join(csrc, "mcpt_sah.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("n,seed,clustered", [(1, 1, 0), (2, 1, 0), (5, 3, 1), (1000, 2, 1), (200000, 4, 0)])
def test_sah_search_tree_invariants(sah_check_exe, n, seed, clustered):
    """The EXACT path's SAH tree (csrc/mcpt_sah.cpp): every reference leaf
    exactly once with its own box, every slot box the exact union of its
    child's, children after parents, the stack bound, and the same bytes for 1
    or 8 build threads (tests/native/sah_check.cpp)."""
    import subprocess
    out = subprocess.run([sah_check_exe, str(n), str(seed), str(clustered)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


# ------------------------------------------------- treelet restructuring
def _sah_metric(nodes):
    """BVH::TEST::SAH (bvhtest.cpp:97-108), in double like the reference."""
    a = nodes["bbmax"][:, :3].astype(np.float64) - nodes["bbmin"][:, :3]
    ar = 2.0 * (a[:, 0] * a[:, 1] + a[:, 0] * a[:, 2] + a[:, 1] * a[:, 2])
    h = len(nodes) >> 1
    return (1.2 * ar[:h].sum() + ar[h:].sum()) / ar[0]


def _check_tree(nodes, n):
    """Every node reached once from root 0, parent links match, leaves stay at
    [n-1, 2n-2] with their triangles, internal boxes = child unions."""
    seen = np.zeros(len(nodes), np.int64)
    stack = [0]
    assert nodes[0]["parent"] == -1
    while stack:
        x = stack.pop()
        seen[x] += 1
        l, r = int(nodes[x]["left"]), int(nodes[x]["right"])
        if l == r:
            assert x >= n - 1
            continue
        assert x < n - 1
        for c in (l, r):
            assert nodes[c]["parent"] == x
            stack.append(c)
        assert (nodes[x]["bbmin"] == np.minimum(nodes[l]["bbmin"], nodes[r]["bbmin"])).all()
        assert (nodes[x]["bbmax"] == np.maximum(nodes[l]["bbmax"], nodes[r]["bbmax"])).all()
    assert (seen == 1).all()


@pytest.mark.parametrize("name", ["cbox", "mis", "random"])
def test_oracle_treelet_is_a_valid_tree_with_lower_sah(name):
    """TreeletBVH<CPU> restated (oracle/mcpt_oracle_treelet.cpp): the rebuilt
    tree is a permutation of the HLBVH's internal nodes over the same leaves,
    and the reference's SAH metric drops (cbox 37.5 -> 28.7, mis 9.4 -> 5.2)."""
    if name == "random":
        rng = np.random.default_rng(3)
        v = rng.uniform(0, 10, (3000, 3, 3)).astype(np.float32)
        t = np.zeros(len(v), L.TRIANGLE)
        t["v"][:, :, :3] = v
        tris = S.pack_triangles(t, np.zeros(len(v), np.int32))
        nodes = S.build_hlbvh(tris)
    else:
        data = getattr(scenes, name)()
        tris, nodes = data.tris, data.nodes
    rc, out = O.treelet(nodes)
    assert rc == 0
    n = len(tris)
    assert (out["left"][n - 1:] == nodes["left"][n - 1:]).all()
    assert (out["bbmin"][n - 1:] == nodes["bbmin"][n - 1:]).all()
    _check_tree(out, n)
    assert _sah_metric(out) < _sah_metric(nodes)
    assert S.bvh_stack_depth(out) <= 64


def test_oracle_treelet_reports_the_reference_recursion_cycle():
    """treeletBVH.cpp:327 reads the first leaf (n-1) as an internal node whose
    children are node `left` (its triangle index).  When that index names an
    ancestor of the leaf, the reference recurses forever; the oracle says -1."""
    n = 40
    x = np.arange(n, dtype=np.float32)  # triangle 0 has the smallest Morton code
    v = np.zeros((n, 3, 3), np.float32)
    v[:, 0, 0], v[:, 1, 0], v[:, 2, 0] = x, x + 0.5, x
    v[:, 2, 1] = 0.5
    t = np.zeros(n, L.TRIANGLE)
    t["v"][:, :, :3] = v
    tris = S.pack_triangles(t, np.zeros(n, np.int32))
    nodes = S.build_hlbvh(tris)
    assert nodes[n - 1]["left"] == 0  # leaf n-1 holds triangle 0 = the root's index
    rc, _ = O.treelet(nodes)
    assert rc == -1


def _random_tree(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.uniform(0, 10, (n, 3, 3)).astype(np.float32)
    t = np.zeros(len(v), L.TRIANGLE)
    t["v"][:, :, :3] = v
    tris = S.pack_triangles(t, np.zeros(len(v), np.int32))
    return tris, S.build_hlbvh(tris)


@pytest.mark.parametrize("name", ["cbox", "mis", "dining", "random"])
def test_oracle_treelet_gpu_is_a_valid_tree_unlike_the_cpu_pass(name):
    """TreeletBVH<GPU> restated (oracle/mcpt_oracle_treelet_gpu.cpp, the tree
    every reference render traverses, scenebuild.cpp:87-95): a permutation of
    the HLBVH's internal nodes over the same leaves, a lower SAH metric, and a
    DIFFERENT tree from TreeletBVH<CPU>'s (array queue with pickNode's argmax,
    reduction-based 6/7-leaf splits, refit without /rootArea)."""
    if name == "random":
        tris, nodes = _random_tree(3000, 3)
    else:
        data = getattr(scenes, name)()
        tris, nodes = data.tris, data.nodes
    rc, out, st = O.treelet_gpu(nodes)
    assert rc == 0
    n = len(tris)
    assert (out["left"][n - 1:] == nodes["left"][n - 1:]).all()
    assert (out["bbmin"][n - 1:] == nodes["bbmin"][n - 1:]).all()
    _check_tree(out, n)
    assert _sah_metric(out) < _sah_metric(nodes)
    assert S.bvh_stack_depth(out) <= 64
    assert st[0] > 0 and st[0] + st[5] == n - 1  # every internal node processed once
    assert st[6] == 0  # no +-0 min/max ties: the v_min/v_max sign rule decides nothing here
    if name != "dining":  # the proxy's leaf n-1 names an ancestor (TreeletBVH<CPU> refuses it)
        rc2, cpu = O.treelet(nodes)
        assert rc2 == 0 and cpu.tobytes() != out.tobytes()


def test_treelet_gpu_missing_root_area_and_lane_rule_decide_the_tree():
    """treeletBVH.cl:524-525 refits without /rootArea: rebuilt nodes carry
    un-normalised costs that later pickNode / DP choices compare with
    normalised ones.  Dividing there (TreeletBVH<CPU>'s :292-293 form) gives a
    different cbox tree; so does letting the LOWEST lane's store land on
    pickNode's maxNodeID / the 6-7-leaf popt (the restatement takes the
    highest).  The quirk counters show each path runs."""
    nodes = scenes.cbox().nodes
    _, base, st = O.treelet_gpu(nodes)
    _, norm, _ = O.treelet_gpu(nodes, options=2)
    _, low, st_low = O.treelet_gpu(nodes, options=1)
    assert base.tobytes() != norm.tobytes()
    assert base.tobytes() != low.tobytes()
    assert st[1] > 0 and st[2] > 0  # several lanes store maxNodeID; none does (stale value kept)
    assert st_low[0] > st[0]  # the lowest-lane rule grows fuller treelets
    # rcp parameter: the correctly rounded reciprocal is the default (bits 0)
    m = O.root_area_mant(nodes)
    r = np.float32(1.0) / m
    _, same, _ = O.treelet_gpu(nodes, rcp_bits=int(r.view(np.uint32)))
    assert same.tobytes() == base.tobytes()


def test_treelet_gpu_argument_checks():
    _, nodes = _random_tree(50, 1)
    swapped = nodes.copy()
    swapped[0]["left"], swapped[0]["right"] = nodes[0]["right"], nodes[0]["left"]
    assert O.treelet_gpu(swapped)[0] == 0  # child order is free
    assert O.treelet_gpu(nodes[:-1])[0] == -2  # even node count
    assert O.treelet_gpu(nodes, options=4)[0] == -2


# ------------------------------------------------------ testbvh metrics
@pytest.mark.parametrize("name", ["cbox", "mis"])
def test_sah_metric_product_equals_oracle(name):
    """BVH::TEST::SAH (bvhtest.cpp:97-108): product (host C++) = oracle (C)."""
    from montecarlopathtracing_amd import bvhtest as B
    nodes = getattr(scenes, name)().nodes
    for nd in (nodes, O.treelet(nodes)[1]):
        assert np.float32(B.sah(nd)) == np.float32(O.bvh_sah(nd))
        assert abs(B.sah(nd) - _sah_metric(nd)) < 1e-5 * _sah_metric(nd)


def test_oracle_lcv_counts_are_leaf_box_hits():
    """LCV's per-ray count (bvhtest.cpp:332-357) = leaves whose box and every
    ancestor's box pass the slab test; checked by brute force on a small tree."""
    rng = np.random.default_rng(9)
    v = rng.uniform(0, 10, (60, 3, 3)).astype(np.float32)
    t = np.zeros(len(v), L.TRIANGLE)
    t["v"][:, :, :3] = v
    nodes = S.build_hlbvh(S.pack_triangles(t, np.zeros(len(v), np.int32)))
    cam = S.parse_camera({"position": [5, 5, -20], "lookat": [5, 5, 0], "up": [0, 1, 0], "fov": 40})
    w, h = 24, 16
    lcv, counts = O.bvh_lcv(nodes, cam, w, h)
    c = cam[0]
    dist = np.float32(0.5) / np.tan(np.float32(c["arg"]) / np.float32(2))
    n = len(v)
    for i in range(w):
        for j in range(h):
            t1 = np.float32((np.float32(i) + np.float32(0.5)) / np.float32(w) - np.float32(0.5))
            t2 = np.float32((np.float32(j) + np.float32(0.5)) / np.float32(h) - np.float32(0.5))
            d = (dist * c["direction"][:3] + t1 * c["horizontal"][:3] + t2 * c["up"][:3]).astype(np.float32)
            o = c["center"][:3].astype(np.float32)
            with np.errstate(divide="ignore", invalid="ignore"):
                def ok(k):
                    a = (nodes[k]["bbmin"][:3] - o) / d
                    b = (nodes[k]["bbmax"][:3] - o) / d
                    tn, tf = np.minimum(a, b).max(), np.maximum(a, b).min()
                    return not (tf < tn or tf < np.float32(0.001))
                want = 0
                for leaf in range(n - 1, 2 * n - 1):
                    k, good = leaf, True
                    while k != -1 and good:
                        good = ok(k)
                        k = nodes[k]["parent"]
                    want += good
            assert counts[i * h + j] == want, (i, j)
    assert lcv == np.float32(np.sqrt((counts.astype(np.float64) ** 2).mean() - counts.mean() ** 2))


@pytest.mark.parametrize("name", ["cbox", "mis"])
def test_oracle_epo_vs_reference_kernel_golden(name):
    """EPO.cl restated in C (fmaf where OpenCL contracts) against the
    reference kernel's own per-triangle output (tests/golden/epo_*.npz,
    tools/make_goldens.py bvh): within 1e-4 relative per triangle (the GPU's
    3-ulp sqrt and 2.5-ulp division vs libm), the metric within 1e-6."""
    import hashlib

    from montecarlopathtracing_amd import bvhtest as B
    path = os.path.join(GOLD, "epo_%s.npz" % name)
    if not os.path.exists(path):
        pytest.skip("golden not generated yet")
    g = np.load(path)
    d, obj = {"cbox": ("scenes/cbox/", "cbox.obj"), "mis": ("scenes/veach_mis/", "mis.obj")}[name]
    tris = B.load_triangles(os.path.join(ROOT, d), obj)
    for bt in ("hlbvh", "treelet"):
        nodes = S.build_hlbvh(tris) if bt == "hlbvh" else O.treelet(S.build_hlbvh(tris))[1]
        assert hashlib.sha1(nodes.tobytes()).digest() == g[bt + "_nodes_sha1"].tobytes()
        e, a = O.bvh_epo(nodes, tris)
        np.testing.assert_allclose(a, g[bt + "_area"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(e, g[bt + "_epo"], rtol=1e-4, atol=1e-3 * float(np.median(g[bt + "_area"])))
        mine = np.sum(e, dtype=np.float64) / np.sum(a, dtype=np.float64)
        ref = np.sum(g[bt + "_epo"], dtype=np.float64) / np.sum(g[bt + "_area"], dtype=np.float64)
        assert abs(mine - ref) <= 1e-6 * ref


def test_diningroom_proxy_is_regenerated_bit_for_bit(tmp_path, monkeypatch):
    """C4's scene is a documented proxy (tools/make_diningroom_proxy.py): the
    committed OBJ is exactly what the generator writes, with the reference's
    diningroom.mtl materials by name and its camera in view."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mkdr", os.path.join(ROOT, "tools", "make_diningroom_proxy.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = tmp_path / "d.obj"
    mod.build().write(str(out))
    assert out.read_bytes() == open(os.path.join(ROOT, "scenes", "diningroom", "diningroom.obj"), "rb").read()
    tris, mats, idx = S.load_object(os.path.join(ROOT, "scenes", "diningroom") + "/", "diningroom.obj")
    assert 90_000 < len(tris) < 110_000
    assert sorted(set(mats["type"].tolist())) == [L.MCPT_DIFFUSE, L.MCPT_GLOSSY, L.MCPT_LIGHT]
    assert (idx >= 0).all()


# ------------------------------------------------------------- sanitizers
@pytest.mark.parametrize("variant", ["host_asan", "host_tsan"])
def test_host_code_under_sanitizers(variant):
    """The host half of libmcpt_hip.so (csrc/mcpt_host.cpp: loader, packing,
    HLBVH, stack depth, SAH metric, camera, classification, RGBE writer;
    csrc/mcpt_sah.cpp: the multi-threaded SAH search-tree builder) on the
    committed scenes, synthetic meshes and edge cases, built with
    AddressSanitizer + UndefinedBehaviorSanitizer (no recovery) and with
    ThreadSanitizer (tests/native/host_sanitize.cpp)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    native = os.path.join(root, "tests", "native")
    subprocess.run(["make", "-s", "-C", native, variant], check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(native, variant), root, "8"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("0 failures"), r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


# ------------------------------------------- the reference's own host C++
# tests/golden/ref_host.npz: outputs of the reference's unmodified host code
# (auxiliary.cpp, thirdpartywrapper.cpp, BVH/treeletBVH.cpp, bvhtest.cpp)
# compiled by oracle/Makefile and run by tools/make_host_goldens.py.
def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


HOST_TREES = {"cbox": lambda: scenes.cbox().nodes, "mis": lambda: scenes.mis().nodes,
              "random20k": lambda: S.random_mesh(20_000, seed=11).nodes}


def test_parse_camera_equals_reference_host():
    """mcpt_parse_camera == Auxiliary::parseCamera (auxiliary.cpp:20-71), the
    reference's own compiled code, bit for bit on the scenes' cameras and 24
    random ones."""
    g = gold("ref_host.npz")
    for inp, rec in zip(g["camera_inputs"], g["cameras"]):
        c = {"position": list(inp[0:3]), "lookat": list(inp[3:6]), "up": list(inp[6:9]), "fov": float(inp[9])}
        assert S.parse_camera(c).tobytes() == rec.tobytes(), c


@pytest.mark.parametrize("name,d,obj", [("cbox", "scenes/cbox/", "cbox.obj"), ("mis", "scenes/veach_mis/", "mis.obj"),
                                        ("dining", "scenes/diningroom/", "diningroom.obj")])
def test_load_object_equals_reference_host(name, d, obj):
    """mcpt_load_obj == ThirdPartyWrapper::loadObject (thirdpartywrapper.cpp:25-99):
    the same Triangle[] and matId[] bytes and the same classified Material[]
    records as the reference's own loader (tinyobj + its material rules)."""
    g = gold("ref_host.npz")
    t, m, i = S.load_object(os.path.join(ROOT, d), obj)
    assert len(t) == int(g["load_%s_n" % name])
    assert _sha(t) == str(g["load_%s_tris_sha" % name])
    assert _sha(i) == str(g["load_%s_ids_sha" % name])
    assert m.tobytes() == g["load_%s_mats" % name].tobytes()


@pytest.mark.parametrize("name", sorted(HOST_TREES))
def test_treelet_and_sah_equal_reference_host(name):
    """The treelet restatement (oracle/mcpt_oracle_treelet.cpp, which the GPU
    pass equals) == TreeletBVH<CPU> (treeletBVH.cpp:30-372) compiled from the
    reference, byte for byte; mcpt_bvh_sah == BVH::TEST::SAH (bvhtest.cpp:104-115)
    on the HLBVH and the treelet tree."""
    from montecarlopathtracing_amd import bvhtest as B
    g = gold("ref_host.npz")
    nodes = HOST_TREES[name]()
    assert _sha(nodes) == str(g["treelet_%s_in_sha" % name])  # the same input tree
    rc, tl = O.treelet(nodes)
    assert rc == 0 and _sha(tl) == str(g["treelet_%s_out_sha" % name])
    assert np.float32(B.sah(nodes)).view(np.uint32) == g["sah_%s_hlbvh_bits" % name]
    assert np.float32(B.sah(tl)).view(np.uint32) == g["sah_%s_treelet_bits" % name]


def test_lcv_oracle_equals_reference_host():
    """The LCV restatement == BVH::TEST::LCV (bvhtest.cpp:324-444) compiled from
    the reference (cbox, config 2's 256 x 256)."""
    g = gold("ref_host.npz")
    w, h = (int(x) for x in g["lcv_size"])
    v, _ = O.bvh_lcv(scenes.cbox().nodes, S.parse_camera(scenes.CBOX_CAM), w, h)
    assert np.float32(v).view(np.uint32) == g["lcv_cbox_bits"]


def test_png_preview_round_trip(tmp_path):
    """The gamma-2.2 display image as PNG (testkernel.cl's pass, SURVEY §8(f)
    rank 2): 8-bit round(clamp(c, 0, 1) * 255), top row first like the .hdr,
    decoded back bit for bit."""
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(3)
    pv = rng.uniform(-0.2, 1.3, (37, 53, 4)).astype(np.float32)
    pv[0, 0, :3] = [np.nan, np.inf, -np.inf]
    pv[..., 3] = 0.0
    S.write_png(str(tmp_path / "p.png"), pv)
    with PIL.open(tmp_path / "p.png") as im:
        got = np.asarray(im.convert("RGB"))
    want = np.clip(np.nan_to_num(pv[::-1, :, :3], nan=0.0, posinf=1.0, neginf=0.0), 0, 1)
    want = np.floor(want * 255 + 0.5).astype(np.uint8)
    assert got.shape == (37, 53, 3) and np.array_equal(got, want)
    assert np.array_equal(got[-1, 0], [0, 255, 0])  # NaN -> 0, +inf -> 1, -inf -> 0 (bottom row, flipped)


TREELET_CL = "/root/reference/MonteCarloPathTracing/kernels/treeletBVH.cl"


def _cl_table(text, name):
    """The integer initialiser of `__constant const <type> name[...] = {...};`
    in treeletBVH.cl, as nested lists (comments stripped)."""
    import re
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    m = re.search(r"\b%s\s*(\[[^\]]*\])+\s*=\s*(\{.*?\})\s*;" % re.escape(name), text, flags=re.S)
    assert m, name
    body = m.group(2)
    rows = re.findall(r"\{([^{}]*)\}", body[1:-1]) if body.count("{") > 1 else [body[1:-1]]
    return [[int(x) for x in r.replace("\n", " ").split(",") if x.strip()] for r in rows]


@pytest.mark.skipif(not os.path.exists(TREELET_CL), reason="the reference is only in the build container")
def test_treelet_cl_dp_schedule_tables():
    """The DP round tables of the reference's GPU treelet kernel
    (kernels/treeletBVH.cl:193-228), read from the reference itself, hold
    what the restatement (csrc/mcpt_treelet_gpu.hip, oracle/
    mcpt_oracle_treelet_gpu.cpp) assumes of them:
    - roundConstant's five rounds list every 2..5-leaf mask of the 7-leaf
      treelet exactly once, constLen rows long, and every mask comes after
      all of its 2+-leaf subsets (so any order of each mask after its
      subsets computes the same DP);
    - roundSixConstant lists the seven 6-leaf masks; roundSixPart[i] is the
      increasing list of the non-empty subsets of that mask without its
      lowest bit (31 partitions, one per lane);
    - roundSeven lists the 63 even masks 2..126 and leaves entry 63 zero:
      lane 31's second candidate reads copt[0] (assumption A2)."""
    text = open(TREELET_CL).read()
    rc = _cl_table(text, "roundConstant")
    cl = _cl_table(text, "constLen")[0]
    assert [len(r) for r in rc] == cl == [10, 20, 29, 32, 21]
    flat = [m for r in rc for m in r]
    want = sorted(m for m in range(1, 127) if 2 <= bin(m).count("1") <= 5)
    assert sorted(flat) == want and len(flat) == len(set(flat)) == 112
    round_of = {m: k for k, r in enumerate(rc) for m in r}
    for m in flat:  # every 2+-leaf proper subset is in a strictly earlier round
        s = (m - 1) & m
        while s:
            if bin(s).count("1") >= 2:
                assert round_of[s] < round_of[m], (s, m)
            s = (s - 1) & m
    six = _cl_table(text, "roundSixConstant")[0]
    assert six == sorted(m for m in range(127) if bin(m).count("1") == 6) == [63, 95, 111, 119, 123, 125, 126]
    parts = _cl_table(text, "roundSixPart")
    assert len(parts) == 7
    for m, p in zip(six, parts):
        rest = m & ~(m & -m)  # the mask without its lowest bit
        subs = sorted(s for s in range(1, 128) if s & ~rest == 0)
        assert p == subs and len(p) == 31, m
    seven = _cl_table(text, "roundSeven")[0]
    assert seven == list(range(2, 127, 2)) and len(seven) == 63  # 64-entry array: [63] is zero-initialised
    import re
    assert re.search(r"roundSeven\s*\[\s*64\s*\]", text)


def test_integration_snippet_matches_abi_host():
    """INTEGRATION.md's "binding a maintainer would add" makes the C ABI calls
    of the tested binding (tests/native/abi_host.cpp: init, then update up
    to the .hdr dump), in the same order -- the GPU treelet pass over the
    HLBVH included (scenebuild.cpp:87-95; VERDICT r3 weak 1: the snippet
    used to skip it)."""
    import re
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc.split("## The binding a maintainer would add", 1)[1]
    snippet = sec.split("```cpp", 1)[1].split("```", 1)[0]
    src = open(os.path.join(ROOT, "tests", "native", "abi_host.cpp")).read()
    body = src[src.index("OK(mcpt_ctx_create"):]
    body = body[:body.index("OK(mcpt_write_hdr") + 1]
    calls = lambda t: re.findall(r"OK\((mcpt_\w+)\(", t)  # noqa: E731
    want = calls(body) + ["mcpt_write_hdr"]
    assert calls(snippet) == want
    assert "mcpt_treelet_gpu" in want


def _spread_slot(j, items):
    """mcpt_device.hip k_render fetch, pixel_spread on: queue slot j of a queue
    holding items / 64 tiles -> (the queue's tile u, its pixel k)."""
    u, k = j >> 6, j & 63
    g0 = u & ~63
    gs = min(64, (items >> 6) - g0)
    i = ((u - g0) << 6) + k
    return g0 + i % gs, i // gs


@pytest.mark.parametrize("n_tiles", [1, 7, 64, 65, 130, 1000, 16384])
def test_spread_slot_mapping_is_a_bijection(n_tiles):
    """The spread slot mapping (mcpt_tuning.pixel_spread) restated: on every
    queue (tiles x, x + nq, ...; queue_items slots) it is a bijection of the
    queue's slots onto its (tile, pixel) pairs -- partial last groups
    included -- and a run of 64 consecutive slots of a full group takes one
    pixel of each of 64 tiles."""
    for nq in (1, 3, 8):
        for x in range(nq):
            n_q = (n_tiles - 1 - x) // nq + 1 if x < n_tiles else 0
            items = n_q * 64
            got = [_spread_slot(j, items) for j in range(items)]
            assert sorted(got) == [(u, k) for u in range(n_q) for k in range(64)]
            if n_q >= 64:
                assert len({u for u, _ in got[:64]}) == 64


def test_trim_profiles_keeps_the_timed_dispatch(tmp_path):
    """tools/trim_profiles.py: a --pmc pass keeps only the rows of the timed
    dispatch (the last dispatch of the kernel its summary names), a trace only
    the render path's kernels; what tools/profile.py summarises is unchanged."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("trim", os.path.join(ROOT, "tools", "trim_profiles.py"))
    T = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(T)
    k = "void k_render<0, false, false, true, false, false, false, 0>(RenderArgs)"
    kp = "void k_render<0, false, false, true, false, true, false, 0>(RenderArgs)"
    hdr = '"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
    rows = [(1, "__amd_rocclr_fillBufferAligned", "SQ_WAVES", 4), (2, kp, "SQ_WAVES", 10), (3, k, "SQ_WAVES", 20),
            (3, k, "GRBM_GUI_ACTIVE", 30), (4, kp, "SQ_WAVES", 11), (5, k, "SQ_WAVES", 40), (5, k, "GRBM_GUI_ACTIVE", 50)]
    pmc = tmp_path / "rx_pmc_sq.csv"
    pmc.write_text(hdr + "".join('%d,"%s","%s",%d\n' % r for r in rows))
    (tmp_path / "rx_summary.json").write_text(json.dumps({"kernel": k}))
    trace = tmp_path / "rx_kernel_trace.csv"
    trace.write_text('"Dispatch_Id","Kernel_Name"\n1,"__amd_rocclr_copyBuffer"\n2,"%s"\n3,"k_tile_sort(x)"\n' % k)
    T.main([str(pmc), str(trace)])
    import csv
    kept = list(csv.DictReader(open(pmc)))
    assert [(int(r["Dispatch_Id"]), r["Counter_Name"], float(r["Counter_Value"])) for r in kept] == \
        [(5, "SQ_WAVES", 40.0), (5, "GRBM_GUI_ACTIVE", 50.0)]
    assert [r["Kernel_Name"] for r in csv.DictReader(open(trace))] == [k, "k_tile_sort(x)"]


def test_td_floor_fit_is_recomputable():
    """profiles/td_floor_fit.json is what tools/profile.py refit computes from
    the committed summaries, and the bench line's TD fields stay fractions:
    every pmc_summary.json entry's TD busy per cycle is at most 1."""
    fit = json.load(open(os.path.join(ROOT, "profiles", "td_floor_fit.json")))
    assert fit["profiles"] >= 35 and fit["a_cycles_per_gather_inst"] > 0 and fit["c_cycles_per_l2_request"] > 0
    for wl, (lo, hi) in fit["range_by_workload"].items():
        assert 0 < lo <= hi < 1.1, (wl, lo, hi)
    # the model accounts for TD's busy cycles where the kernel is bound by its
    # gathers; where VALU is saturated (round 6's C3, VALU busy >= 1) TD's
    # busy count also holds data waiting on the busy VGPR write port, which no
    # gather term models, so only the upper bound applies there
    for tag, r in fit["modelled_over_measured_busy"].items():
        summ = json.load(open(os.path.join(ROOT, "profiles", "%s_summary.json" % tag)))
        if summ["valu_busy"] < 0.95:
            assert 0.7 < r < 1.1, (tag, r)
    entries = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
    for key, e in entries.items():
        summ = json.load(open(os.path.join(ROOT, e["source"])))
        c = summ["counters_timed_dispatch"]
        busy = c["TD_TD_BUSY_sum"] / (summ.get("cus", 256) * summ["kernel_cycles"])
        assert abs(busy - e["td_fit"]["td_busy_per_cycle"]) < 1e-3 and busy <= 1.0, key
        floor = (fit["a_cycles_per_gather_inst"] * c["SQ_INSTS_VMEM_RD"] + fit["b_cycles_per_l1_hit_line"] *
                 (c["TCP_TOTAL_CACHE_ACCESSES_sum"] - c["TCP_TCC_READ_REQ_sum"]) +
                 fit["c_cycles_per_l2_request"] * c["TCP_TCC_READ_REQ_sum"]) / summ.get("cus", 256)
        assert abs(floor / summ["kernel_cycles"] - e["td_fit"]["model_frac"]) < 2e-3, key


def test_bench_strong_record():
    """bench.strong_record: the striped rate, every rank's share time, and the
    speed-up over the same image rendered on one GPU inside the job."""
    import bench
    bench.DEPTH = 8
    r = bench.strong_record(1024, 1024, 20, 0.004, [0.003, 0.004], 0.0092, "n")
    assert r["value"] == round(1024 * 1024 * 20 * 8 / 0.004 / 1e6, 2)
    assert r["share_ms_per_rank"] == [3.0, 4.0] and r["share_max_over_mean"] == round(4 / 3.5, 4)
    assert r["one_gpu_ms"] == 9.2 and r["speedup_vs_1gpu"] == 2.3
    assert bench.strong_record(8, 8, 1, 1.0, [1.0], None, "n")["speedup_vs_1gpu"] is None


def test_variant_names_map_to_macros(tmp_path):
    """`make variants` (the A/B builds tools/ab.py and tools/sweep.py time):
    each letter of a variant name sets its macro, the rest keep the shipped
    values (dry run: the compiler is `echo`)."""
    import subprocess
    out = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "montecarlopathtracing_amd", "csrc"), "variants",
                          "VARIANTS=w4k16 w5l0 w5g1", "HIPCC=echo", "OUT=%s" % tmp_path],
                         capture_output=True, text=True, check=True).stdout
    lines = [ln for ln in out.splitlines() if "mcpt_device.hip" in ln]
    assert len(lines) == 3
    macros = [dict(re.findall(r"-D(MCPT_[A-Z_]+)=(\S+)", ln)) for ln in lines]
    shipped = {"MCPT_STACK_WINDOW_K": "16", "MCPT_POW_LOBE": "1", "MCPT_WG_WAVES": "4"}
    assert macros[0] == dict(shipped, MCPT_WAVES_PER_SIMD="4")
    assert macros[1] == dict(shipped, MCPT_WAVES_PER_SIMD="5", MCPT_POW_LOBE="0")
    assert macros[2] == dict(shipped, MCPT_WAVES_PER_SIMD="5", MCPT_WG_WAVES="1")


def test_bench_refuses_more_ranks_than_gpus():
    """bench.py at WORLD_SIZE > visible GPUs (one rank per GPU) exits non-zero
    before any call that initialises a device, and does not re-launch itself:
    here (no GPU) two ranks see zero devices."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29555")
    env.pop("MCPT_BENCH_SHARED_GPU", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr[-2000:]
    assert "needs 2 visible GPUs" in r.stderr and not r.stdout.strip()
