"""Time mcpt_scene_upload_device alone (the scene already in HBM: HLBVH and
the GPU treelet pass done first), for rocprofv3 runs of the upload kernels.

    python tools/upload_probe.py [C2 C5 ...] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import load_scene  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["C2", "C5"])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    rnd = R.Renderer(0)
    for wl in a.workloads:
        data, _ = load_scene(wl)
        dt = R.to_device(data.tris, 0)
        dn = R.build_hlbvh_device(dt)
        R.treelet_gpu_device(dn)
        rnd.upload((dt, dn, data.mats)).close()  # warm
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sc = rnd.upload((dt, dn, data.mats))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            meta = sc.read("meta").tolist()
            sc.close()
        print(json.dumps({"workload": wl, "triangles": len(data.tris), "upload_device_s": [round(t, 4) for t in ts],
                          "meta": meta}), flush=True)
    rnd.close()


if __name__ == "__main__":
    main()
