#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

* gpu part (run on the MI355X box; needs oracle/_ref built here first):
  the reference's own OpenCL kernels compiled for gfx950 (tests/refgpu.py)
  produce rays, hits, shade transitions, accumulation steps and whole images
  on seeded inputs.
* cpu part (run here; needs /root/reference): the reference's vendored
  tinyobjloader and stb_image_write (oracle/_ref/libref_io.so) load the
  committed scenes and encode images.

    python tools/make_goldens.py gpu  OUTDIR
    python tools/make_goldens.py cpu  OUTDIR
    python tools/make_goldens.py bvh  OUTDIR   (GPU box: EPO.cl per triangle)
    python tools/make_goldens.py app  OUTDIR   (GPU box: C1 over the GPU-treelet tree)
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import scenes  # noqa: E402

CAMS = {"cbox": scenes.CBOX_CAM, "mis": scenes.MIS_CAM, "dining": scenes.DINING_CAM}


def gpu(out):
    from tests import refgpu
    os.makedirs(out, exist_ok=True)
    # (1) generateRay, 64x48, three cameras
    rays = {k: refgpu.generate(S.parse_camera(c), 64, 48) for k, c in CAMS.items()}
    np.savez_compressed(os.path.join(out, "rays.npz"), **{k: v.view(np.uint8) for k, v in rays.items()})
    # (2)+(3) bounce chains: inputs and outputs of intersect and shade, per bounce
    for name, getter, cam in (("cbox", scenes.cbox, scenes.CBOX_CAM), ("mis", scenes.mis, scenes.MIS_CAM)):
        data = getter()
        w, h, depth = 48, 40, 6
        r = refgpu.generate(S.parse_camera(cam), w, h)
        n = len(r)
        seeds = R.default_seeds(n)
        col = np.ones((n, 4), np.float32)
        hits = np.zeros(n, L.HIT)
        rec = {}
        for b in range(depth):
            rec["rays%d" % b] = r.view(np.uint8).copy()
            rec["hits_in%d" % b] = hits.view(np.uint8).copy()
            hits = refgpu.intersect(data, r, hits=hits)
            rec["hits%d" % b] = hits.view(np.uint8).copy()
            rec["colors_in%d" % b] = col.copy()
            rec["seeds_in%d" % b] = seeds.copy()
            r, col, seeds = refgpu.shade(data, r, hits, col, seeds, depth)
            rec["rays_out%d" % b] = r.view(np.uint8).copy()
            rec["colors%d" % b] = col.copy()
            rec["seeds%d" % b] = seeds.copy()
        rec["depth"] = np.int32(depth)
        np.savez_compressed(os.path.join(out, "chain_%s.npz" % name), **rec)
    # (4) history.cl on random colours
    rng = np.random.default_rng(7)
    w, h, att = 32, 16, 8
    hist = np.zeros((w * h, 4), np.float32)
    cnt = np.zeros(w * h, np.int32)
    acc = {}
    for f in range(att + 2):
        c = rng.exponential(1.0, (w * h, 4)).astype(np.float32)
        c[rng.random(w * h) < 0.3] = 0.0
        c[:, 3] = 0.0
        acc["in%d" % f] = c
        c2, hist, cnt = refgpu.accumulate(c, hist, cnt, w, h, att)
        acc["disp%d" % f], acc["hist%d" % f], acc["count%d" % f] = c2, hist, cnt
    np.savez_compressed(os.path.join(out, "accumulate.npz"), **acc)
    # (5) whole images: C1 (cbox 256^2, 16 frames, depth 4, attempt 16) and small mis / diffuse cbox
    imgs = [("c1_cbox", scenes.cbox, scenes.CBOX_CAM, 256, 256, 4, 16, 16),
            ("mis64", scenes.mis, scenes.MIS_CAM, 64, 64, 12, 8, 8),
            ("cboxdiff64", scenes.cbox_diffuse, scenes.CBOX_CAM, 64, 64, 8, 8, 8)]
    for name, getter, cam, w, h, depth, frames, att in imgs:
        seeds = R.default_seeds(w * h)
        hh, cc, ss = refgpu.render(getter(), S.parse_camera(cam), w, h, depth, frames, att, seeds)
        np.savez_compressed(os.path.join(out, "image_%s.npz" % name), hist=hh, count=cc, seeds=ss,
                            seeds_in=seeds, meta=np.array([w, h, depth, frames, att], np.int32))
    print("gpu goldens written to", out)


def bvh(out):
    """The reference's EPO.cl kernel (bvhtest.cpp:288-321) per triangle on the
    cbox / veach_mis HLBVH and treelet trees (testbvh's loadObj triangles:
    vertices only)."""
    from montecarlopathtracing_amd import bvhtest as B
    from tests import refgpu
    os.makedirs(out, exist_ok=True)
    for name, d, obj in (("cbox", "scenes/cbox/", "cbox.obj"), ("mis", "scenes/veach_mis/", "mis.obj")):
        tris = B.load_triangles(os.path.join(ROOT, d), obj)
        rec = {}
        for bt in ("hlbvh", "treelet"):
            nodes = B.build(tris, bt)
            e, a = refgpu.epo(nodes, tris)
            rec[bt + "_nodes_sha1"] = np.frombuffer(hashlib.sha1(nodes.tobytes()).digest(), np.uint8)
            rec[bt + "_epo"], rec[bt + "_area"] = e, a
        np.savez_compressed(os.path.join(out, "epo_%s.npz" % name), **rec)


def app(out):
    """C1 as the reference APPLICATION renders it: SceneCL restructures a fresh
    HLBVH with the GPU treelet kernel for every bvhtype (scenebuild.cpp:87-95).
    The tree is the CPU restatement of treeletBVH.cl (oracle/
    mcpt_oracle_treelet_gpu.cpp, fed this GPU's v_rcp_f32), the image the
    reference's own kernels over it (tests/refgpu.py), for the splitmix seeds
    of image_c1_cbox.npz and MSVC rand()'s 15-bit variant of them."""
    from tests import oracle as O
    from tests import refgpu
    os.makedirs(out, exist_ok=True)
    data = scenes.cbox()
    rcp = int(refgpu.rcp_f32(O.root_area_mant(data.nodes))[0].view(np.uint32))
    rc, nodes, _ = O.treelet_gpu(data.nodes, rcp_bits=rcp)
    assert rc == 0
    data = data.with_nodes(nodes)
    w, h, depth, frames, att = 256, 256, 4, 16, 16
    rec = {"meta": np.array([w, h, depth, frames, att], np.int32), "rcp_bits": np.uint32(rcp),
           "nodes_sha256": hashlib.sha256(nodes.tobytes()).hexdigest()}
    for tag, variant in (("", "splitmix"), ("15", "msvc15")):
        seeds = R.default_seeds(w * h, variant=variant)
        hh, cc, ss = refgpu.render(data, S.parse_camera(scenes.CBOX_CAM), w, h, depth, frames, att, seeds)
        rec.update({"hist" + tag: hh, "count" + tag: cc, "seeds" + tag: ss, "seeds_in" + tag: seeds})
    np.savez_compressed(os.path.join(out, "image_c1_app.npz"), **rec)
    print("app golden written to", out)


def cpu(out):
    """Reference tinyobj + stb fixtures (oracle/_ref/libref_io.so)."""
    so = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_io.so"))
    os.makedirs(out, exist_ok=True)
    meta = {}
    for d, obj in (("cbox", "cbox.obj"), ("veach_mis", "mis.obj"), ("diningroom", "diningroom.obj")):
        dirp = os.path.join(ROOT, "scenes", d) + "/"
        nt, nm = ctypes.c_int64(0), ctypes.c_int32(0)
        so.ref_load_obj(dirp.encode(), obj.encode(), None, None, ctypes.byref(nt), None, ctypes.byref(nm))
        v = np.zeros((nt.value, 9), np.float32)
        mi = np.zeros(nt.value, np.int32)
        m = np.zeros((nm.value, 11), np.float32)
        so.ref_load_obj(dirp.encode(), obj.encode(), L.ptr(v), L.ptr(mi), ctypes.byref(nt), L.ptr(m), ctypes.byref(nm))
        np.savez_compressed(os.path.join(out, "tinyobj_%s.npz" % d), verts=v, matids=mi, mtl=m)
        meta[d] = {"triangles": int(nt.value), "materials": int(nm.value),
                   "verts_sha256": hashlib.sha256(v.tobytes()).hexdigest()}
    # stb RGBE bytes: a synthetic image exercising runs, dumps, zeros and large values
    rng = np.random.default_rng(3)
    img = rng.exponential(2.0, (37, 53, 4)).astype(np.float32)
    img[5:9] = 0.0
    img[10, :, :3] = 1.5
    img[12, 3:40, :3] = [0.25, 7.0, 1e-33]
    img[14] = 1e6
    for name, im in (("synthetic", img), ("narrow", img[:, :6].copy())):
        p = os.path.join(out, "stb_%s.hdr" % name)
        so.ref_write_hdr(p.encode(), im.shape[1], im.shape[0], L.ptr(np.ascontiguousarray(im)), 1)
        np.save(os.path.join(out, "stb_%s_input.npy" % name), im)
    with open(os.path.join(out, "cpu_fixtures.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print("cpu goldens written to", out)


if __name__ == "__main__":
    mode, out = sys.argv[1], sys.argv[2]
    {"gpu": gpu, "cpu": cpu, "bvh": bvh, "app": app}[mode](out)
