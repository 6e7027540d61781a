"""BVH::TEST — the reference's "testbvh" / "testall" modes (MCPT/bvhtest.cpp:448-649,
MCPT/main.cpp:14-19) on the HIP path: build the configured BVH for an OBJ and
print its quality metrics.

    SAH      bvhtest.cpp:97-108   host (mcpt_bvh_sah)
    EPO_GPU  bvhtest.cpp:288-321  GPU, kernels/EPO.cl restated (mcpt_bvh_epo_device)
    LCV      bvhtest.cpp:324-444  GPU (mcpt_bvh_lcv_device), when the config has a camera

The BVH is the reference's (bvhtest.cpp:458-519): HLBVH<CPU> (host build,
hlbvh.cpp) for "hlbvh"; TreeletBVH<CPU>'s pass over it for "treelet" (run on
the GPU); the GPU treelet kernel's pass, TreeletBVH<GPU>
(treeletBVH.cl), for "treeletGPU".
Output lines follow the reference's std::cout lines.
"""
import ctypes
import os

import numpy as np

from . import _lib as L
from . import config as C
from . import scene as S


def load_triangles(directory, objname):
    """bvhtest.cpp:47-83 loadObj: the OBJ's triangles, vertices only (the
    render loader's order; normals and material ids stay zero)."""
    tris, _, _ = S.load_object(directory, objname)
    return tris


def build(tris, bvhtype="hlbvh", device=0):
    nodes = S.build_hlbvh(tris)
    if bvhtype == "treelet":
        from . import render as R
        nodes = R.treelet_device(nodes, device)
    elif bvhtype == "treeletGPU":
        from . import render as R
        nodes = R.treelet_gpu_device(nodes, device)
    elif bvhtype != "hlbvh":
        raise ValueError("BVH Not Implemented: %r" % bvhtype)
    return nodes


def sah(nodes):
    out = ctypes.c_double(0.0)
    L.check(L.lib().mcpt_bvh_sah(L.ptr(np.ascontiguousarray(nodes)), len(nodes), ctypes.byref(out)))
    return out.value


def epo(nodes, tris, device=0, per_triangle=False):
    """EPO_GPU: float result; with per_triangle, also the kernel's per-leaf
    EPO and triangle areas and the count of clip-polygon overflows."""
    import torch

    from . import render as R
    n = len(tris)
    dn = R.to_device(nodes, device)
    dt = R.to_device(tris, device)
    e = torch.empty(n, dtype=torch.float32, device=dn.device)
    a = torch.empty(n, dtype=torch.float32, device=dn.device)
    out, ovf = ctypes.c_double(0.0), ctypes.c_uint64(0)
    L.check(L.lib().mcpt_bvh_epo_device(L.ptr(dn), L.ptr(dt), n, L.ptr(e), L.ptr(a), ctypes.byref(out),
                                        ctypes.byref(ovf), R._stream()))
    if per_triangle:
        return out.value, e.cpu().numpy(), a.cpu().numpy(), ovf.value
    return out.value


def lcv(nodes, camera, width, height, device=0, counts=False):
    """LCV: float result; with counts, also the per-ray leaf counts (i*H + j)."""
    import torch

    from . import render as R
    dn = R.to_device(nodes, device)
    c = torch.empty(width * height, dtype=torch.int32, device=dn.device)
    out = ctypes.c_double(0.0)
    cam = np.ascontiguousarray(camera)
    L.check(L.lib().mcpt_bvh_lcv_device(L.ptr(dn), len(nodes), L.ptr(cam), int(width), int(height), L.ptr(c),
                                        ctypes.byref(out), R._stream()))
    if counts:
        return out.value, c.cpu().numpy().view(np.uint32)
    return out.value


def _fmt(x):
    return "%g" % x  # std::cout's default 6 significant digits


def testmodel(directory, objname, bvhtype, camera_json=None, width=0, height=0, device=0, out=print):
    """bvhtest.cpp:448-530 test() / :533-611 testmodel()."""
    tris = load_triangles(directory, objname)
    out("%s %d" % (objname, len(tris)))
    out(bvhtype)
    nodes = build(tris, bvhtype, device)
    res = {"objname": objname, "triangles": len(tris), "bvhtype": bvhtype, "SAH": sah(nodes)}
    out("SAH: " + _fmt(res["SAH"]))
    res["EPO_GPU"] = epo(nodes, tris, device)
    out("EPO_GPU: " + _fmt(res["EPO_GPU"]))
    if camera_json:
        res["LCV"] = lcv(nodes, S.parse_camera(camera_json), width, height, device)
        out("LCV: " + _fmt(res["LCV"]))
    return res


def run(cfg, configid=None, root=".", device=0, out=print):
    """main.cpp:14-19: testall -> every objname of the entry (no camera,
    bvhtest.cpp:633-647); testbvh -> the one model, LCV over its camera."""
    cfg = cfg if isinstance(cfg, C.Config) else C.Config(cfg, configid)
    directory = os.path.join(root, cfg.GETDIRECTORY())
    if not directory.endswith("/"):
        directory += "/"
    if cfg.TESTALL():
        results = []
        for obj in cfg.GETOBJS():
            results.append(testmodel(directory, obj, cfg.BVHTYPE(), None, 0, 0, device, out))
            out("")
        return results
    if not cfg.TESTBVH():
        raise ValueError("config entry is not a testbvh/testall entry")
    return [testmodel(directory, cfg.GETOBJNAME(), cfg.BVHTYPE(), cfg.GETCAMERA(), cfg.WIDTH(), cfg.HEIGHT(), device,
                      out)]
