"""The CPU baseline of every workload: bench.py's cpu_baseline
leg -- the CPU oracle (oracle/mcpt_oracle.c, the reference's exhaustive
traversal) on the process's CPU share over a bounded pixel sample, ~15 s each --
for C1-C5, one JSON line per workload.  Run on the GPU box (its host cores):

    python tools/cpu_baseline.py [C1 C2 C3 C4 C5] > profiles/r02_cpu_baseline.jsonl

C1 is the reference's own CPU-runnable case (cbox 256x256, depth 4)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402

C1 = {"desc": "C1: cbox 256x256, 4 bounces", "w": 256, "h": 256, "depth": 4}


def main():
    for name in sys.argv[1:] or ["C1", "C2", "C3", "C4", "C5"]:
        wl = C1 if name == "C1" else bench.WORKLOADS[name]
        bench.W, bench.DEPTH = wl["w"], wl["depth"]
        if name == "C1":  # the cbox as loaded (all materials), as config.json's configid 2
            from tests import scenes
            data, camj = scenes.cbox(), scenes.CBOX_CAM
        else:
            data, camj = bench.load_scene(name)
            if data.nodes is None:  # C5: the deployed tree, built on the GPU
                from montecarlopathtracing_amd import render as R
                from montecarlopathtracing_amd import _lib as L
                dn = R.build_hlbvh_device(R.to_device(data.tris, 0))
                data = data.with_nodes(R.records(R.treelet_gpu_device(dn), L.BVHNODE).copy())
        cb = bench.cpu_baseline(data, S.parse_camera(camj), wl["h"], label=name)
        print(json.dumps({"workload": wl["desc"], "cpu_baseline": cb}), flush=True)


if __name__ == "__main__":
    main()
