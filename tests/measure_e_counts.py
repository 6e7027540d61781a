"""Measure SURVEY.md §8(d)'s E_node / E_tri per config with the CPU oracle:
mean node visits and triangle tests per active segment of a t-pruned,
left-first traversal of the reference HLBVH (1 box test per 64-B node, as
the reference fetches them).  Writes profiles/e_counts.json (committed; read
by bench.py).  Test infrastructure: run here, not on the GPU box.

    python tests/measure_e_counts.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import oracle as O  # noqa: E402
from tests import scenes  # noqa: E402

def _treelet(nodes):
    rc, out = O.treelet(nodes)
    assert rc == 0, "treelet pass refused this tree"
    return out


CONFIGS = {
    "C1": (scenes.cbox, scenes.CBOX_CAM, 256, 256, 4),
    "C2": (scenes.cbox_diffuse, scenes.CBOX_CAM, 1024, 1024, 8),
    "C3": (scenes.mis, scenes.MIS_CAM, 1024, 1024, 12),
    # C4 renders over the treelet tree (config "bvhtype": "treeletGPU", as the reference's diningroom entry)
    "C4": (lambda: scenes.dining().with_nodes(_treelet(scenes.dining().nodes)), scenes.DINING_CAM, 1920, 1080, 16),
    "C5": (lambda: S.random_mesh(10_000_000), S.RANDOM_MESH_CAMERA, 2048, 2048, 8),
}


def measure(getter, camj, w, h, depth, npix=4096, frames=4, prune=True):
    data = getter()
    cam = S.parse_camera(camj)
    rng = np.random.default_rng(0)
    px = np.sort(rng.choice(w * h, min(npix, w * h), replace=False)).astype(np.int32)
    _, _, _, st = O.render(data, cam, w, h, depth, frames, 1 << 20, R.default_seeds(w * h), pixels=px,
                           prune=prune)
    return {"E_node": float(st[1]) / float(st[0]), "E_tri": float(st[2]) / float(st[0]),
            "segments": int(st[0]), "segments_per_path": float(st[0]) / (len(px) * frames),
            "sample": "%d random pixels x %d frames, %s traversal" % (len(px), frames,
                                                                      "t-pruned" if prune else "exhaustive")}


def main():
    path = os.path.join(ROOT, "profiles", "e_counts.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    only = sys.argv[1:] or list(CONFIGS)
    for k, args in CONFIGS.items():
        if k not in only:
            continue
        out[k] = measure(*args)
        out[k + "_exhaustive"] = measure(*args, prune=False)
        e = out[k]
        e["B_seg"] = 328.0 + 64.0 * (e["E_node"] + e["E_tri"])
        print(k, json.dumps(out[k]), "exhaustive:", json.dumps(out[k + "_exhaustive"]))
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "e_counts.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
