"""Golden fixtures from the reference's OWN host C++ (oracle/_ref/ref_host_golden,
built by `make -C oracle ref` from the unmodified sources under /root/reference):

    python tools/make_host_goldens.py      # writes tests/golden/ref_host.npz

  cameras    Auxiliary::parseCamera (auxiliary.cpp:20-71) of the scenes' cameras
             and 24 random ones: the 80-B Camera records
  load_*     ThirdPartyWrapper::loadObject (thirdpartywrapper.cpp:25-99) of cbox,
             veach_mis and the diningroom proxy: triangle count, SHA-256 of the
             Triangle[] and matId[] bytes, the Material[] records (classification)
  treelet_*  TreeletBVH<CPU> (treeletBVH.cpp:30-372) of the HLBVH of cbox,
             veach_mis and a 20 K random mesh: SHA-256 of the input and output
             BVHNode[] bytes
  sah_*      BVH::TEST::SAH (bvhtest.cpp:104-115) of those trees (float bits)
  lcv_*      BVH::TEST::LCV (bvhtest.cpp:324-444) of cbox at config.json's
             configid entry size (256 x 256, config 2) (float bits)

Run in the build container only (the reference never travels to the GPU box);
the HLBVH inputs come from this repo's host build (BVH/hlbvh.cpp itself does
not compile outside MSVC).  TEST INFRASTRUCTURE.
"""
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import scenes  # noqa: E402

EXE = os.path.join(ROOT, "oracle", "_ref", "ref_host_golden")


def run(*args):
    r = subprocess.run([EXE] + [str(a) for a in args], cwd=ROOT, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit("ref_host_golden %s failed: %s" % (args[0], r.stderr))
    return r.stdout.strip()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def cameras():
    rng = np.random.default_rng(3)
    cams = [scenes.CBOX_CAM, scenes.MIS_CAM, scenes.DINING_CAM, S.RANDOM_MESH_CAMERA]
    for _ in range(24):
        p = rng.uniform(-500, 500, 3)
        la = p + rng.normal(0, 50, 3)
        up = rng.normal(0, 1, 3)
        cams.append({"position": p.tolist(), "lookat": la.tolist(), "up": up.tolist(),
                     "fov": float(rng.uniform(10, 120))})
    return cams


def main():
    if not os.path.exists(EXE):
        raise SystemExit("build oracle/_ref/ref_host_golden first: make -C oracle ref")
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        cams = cameras()
        recs = []
        for c in cams:
            f = os.path.join(tmp, "cam.bin")
            args = list(c["position"]) + list(c["lookat"]) + list(c["up"]) + [c["fov"]]
            run("camera", f, *["%.17g" % float(x) for x in args])
            recs.append(np.fromfile(f, L.CAMERA)[0])
        out["camera_inputs"] = np.array([list(c["position"]) + list(c["lookat"]) + list(c["up"]) + [c["fov"]]
                                         for c in cams], np.float64)
        out["cameras"] = np.array(recs, L.CAMERA)
        for name, d, obj in (("cbox", "scenes/cbox/", "cbox.obj"), ("mis", "scenes/veach_mis/", "mis.obj"),
                             ("dining", "scenes/diningroom/", "diningroom.obj")):
            ft, fm, fi = (os.path.join(tmp, x) for x in ("t.bin", "m.bin", "i.bin"))
            run("load", d, obj, ft, fm, fi)
            tris = np.fromfile(ft, L.TRIANGLE)
            ids = np.fromfile(fi, np.int32)
            out["load_%s_n" % name] = np.int64(len(tris))
            out["load_%s_tris_sha" % name] = sha(tris)
            out["load_%s_ids_sha" % name] = sha(ids)
            out["load_%s_mats" % name] = np.fromfile(fm, L.MATERIAL)
        trees = {"cbox": scenes.cbox().nodes, "mis": scenes.mis().nodes,
                 "random20k": S.random_mesh(20_000, seed=11).nodes}
        for name, nodes in trees.items():
            fin, fout = os.path.join(tmp, "in.bin"), os.path.join(tmp, "out.bin")
            np.ascontiguousarray(nodes).tofile(fin)
            run("treelet", fin, fout)
            tl = np.fromfile(fout, L.BVHNODE)
            out["treelet_%s_in_sha" % name] = sha(nodes)
            out["treelet_%s_out_sha" % name] = sha(tl)
            out["sah_%s_hlbvh_bits" % name] = np.uint32(int(run("sah", fin)))
            out["sah_%s_treelet_bits" % name] = np.uint32(int(run("sah", fout)))
        cbox_nodes = os.path.join(tmp, "cbox.bin")
        np.ascontiguousarray(trees["cbox"]).tofile(cbox_nodes)
        cam = os.path.join(tmp, "cbcam.bin")
        np.ascontiguousarray(S.parse_camera(scenes.CBOX_CAM)).tofile(cam)
        out["lcv_cbox_bits"] = np.uint32(int(run("lcv", cbox_nodes, cam)))
        out["lcv_size"] = np.array([256, 256], np.int32)  # config.json configid 2 (Config::WIDTH/HEIGHT)
    path = os.path.join(ROOT, "tests", "golden", "ref_host.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, "(%d keys)" % len(out))


if __name__ == "__main__":
    main()
