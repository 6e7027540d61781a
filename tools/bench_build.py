"""Scene build times (build time is excluded from the render
metric but reported): the reference HLBVH on the host (mcpt_build_hlbvh, the
restated hlbvh.cpp) vs on the GPU (mcpt_build_hlbvh_device, same bits), and
mcpt_scene_upload (device copies + the EXACT path's SAH search tree), and the
treelet pass ("bvhtype": "treelet") on the GPU vs the CPU oracle's sequential
restatement of TreeletBVH<CPU> (the reference's own algorithm, single thread),
and the GPU treelet kernel's pass every render runs (TreeletBVH<GPU>,
mcpt_treelet_gpu_device) vs its sequential CPU restatement.

    python tools/bench_build.py [C2 C5 ...]  -> one JSON line per workload
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import load_scene  # noqa: E402
from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402


def main():
    for wl in sys.argv[1:] or ["C2", "C5"]:
        data, _ = load_scene(wl)
        tris = data.tris
        t0 = time.perf_counter()
        host = S.build_hlbvh(tris)
        t_host = time.perf_counter() - t0
        dt = R.to_device(tris, 0)
        R.build_hlbvh_device(dt)  # warm (hipCUB kernels, allocator)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev = R.build_hlbvh_device(dt)
        torch.cuda.synchronize()
        t_dev = time.perf_counter() - t0
        same = bool(np.array_equal(R.records(dev, L.BVHNODE).view(np.uint8), host.view(np.uint8)))
        dn = R.build_hlbvh_device(dt)
        R.treelet_device(dn)  # warm
        dn = R.build_hlbvh_device(dt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        R.treelet_device(dn)
        torch.cuda.synchronize()
        t_tl = time.perf_counter() - t0
        t_tl_cpu, tl_same = None, None
        try:
            sys.path.insert(0, ROOT)
            from tests import oracle as O
            if O.available():
                t0 = time.perf_counter()
                rc, ref = O.treelet(host)
                t_tl_cpu = time.perf_counter() - t0
                tl_same = bool(rc == 0 and np.array_equal(R.records(dn, L.BVHNODE).view(np.uint8), ref.view(np.uint8)))
        except ImportError:
            pass
        dn = R.build_hlbvh_device(dt)
        R.treelet_gpu_device(dn)  # warm
        dn = R.build_hlbvh_device(dt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        R.treelet_gpu_device(dn)
        torch.cuda.synchronize()
        t_tg = time.perf_counter() - t0
        t_tg_cpu, tg_same = None, None
        try:
            from tests import oracle as O
            from tests import refgpu
            if O.available() and refgpu.available():
                rcp = int(refgpu.rcp_f32(O.root_area_mant(host))[0].view(np.uint32))
                t0 = time.perf_counter()
                rc, ref, _ = O.treelet_gpu(host, rcp_bits=rcp)
                t_tg_cpu = time.perf_counter() - t0
                tg_same = bool(rc == 0 and np.array_equal(R.records(dn, L.BVHNODE).view(np.uint8), ref.view(np.uint8)))
        except ImportError:
            pass
        deployed = data.with_nodes(R.records(dn, L.BVHNODE).copy())
        rnd = R.Renderer(0)
        t0 = time.perf_counter()
        sc = rnd.upload(deployed)
        torch.cuda.synchronize()
        t_up = time.perf_counter() - t0
        # the same structures built on the GPU from the tree in HBM (mcpt_scene_upload_device)
        dn = R.build_hlbvh_device(dt)
        R.treelet_gpu_device(dn)
        sc2 = rnd.upload((dt, dn, data.mats))  # warm (hipCUB kernels, allocator)
        sc2.close()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc2 = rnd.upload((dt, dn, data.mats))
        torch.cuda.synchronize()
        t_upd = time.perf_counter() - t0
        same_up = all(sc.read(k).tobytes() == sc2.read(k).tobytes() for k in R.DeviceScene.ARRAYS + ("meta",))
        # the whole GPU pipeline from triangles in HBM: HLBVH + GPU treelet pass + upload
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dn = R.build_hlbvh_device(dt)
        R.treelet_gpu_device(dn)
        sc3 = rnd.upload((dt, dn, data.mats))
        torch.cuda.synchronize()
        t_pipe = time.perf_counter() - t0
        sc3.close()
        sc2.close()
        sc.close()
        rnd.close()
        print(json.dumps({"workload": wl, "triangles": len(tris), "hlbvh_host_s": round(t_host, 4),
                          "hlbvh_gpu_s": round(t_dev, 4), "gpu_equals_host": same,
                          "scene_upload_s": round(t_up, 4), "scene_upload_device_s": round(t_upd, 4),
                          "upload_device_equals_host": same_up,
                          "gpu_pipeline_s (hlbvh + treelet kernel pass + upload)": round(t_pipe, 4),
                          "treelet_gpu_s": round(t_tl, 4),
                          "treelet_cpu_oracle_s": None if t_tl_cpu is None else round(t_tl_cpu, 4),
                          "treelet_gpu_equals_oracle": tl_same,
                          "treelet_gpu_kernel_pass_s": round(t_tg, 4),
                          "treelet_gpu_kernel_pass_cpu_oracle_s": None if t_tg_cpu is None else round(t_tg_cpu, 4),
                          "treelet_gpu_kernel_pass_equals_oracle": tg_same,
                          "note": "scene_upload = validation + 4-wide trees (reference collapse + SAH search "
                                  "tree, host, 16 threads) + device copies"}), flush=True)


if __name__ == "__main__":
    main()
