"""Child process of tests/test_gpu_debug.py: renders with the MCPT_DEBUG build
of the library (MCPT_LIB_OVERRIDE=.../libmcpt_hip_debug.so) and prints one
JSON line per case with the bounds-check violation count and a digest of the
result.  Test infrastructure."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import scenes  # noqa: E402


def digest(st):
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for a in (st.hist.cpu().numpy(), st.count.cpu().numpy(), st.seeds_np()):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    rnd = R.Renderer(0)
    print(json.dumps({"version": L.lib().mcpt_version().decode()}), flush=True)
    g = np.load(os.path.join(ROOT, "tests", "golden", "image_c1_cbox.npz"))
    w, h, depth, frames, att = (int(x) for x in g["meta"])
    cases = [("c1", scenes.cbox(), scenes.CBOX_CAM, w, h, depth, frames, att, g["seeds_in"], {}),
             ("dining", scenes.dining(), scenes.DINING_CAM, 96, 64, 16, 4, 4, None, {}),
             ("c5_window", S.random_mesh(500_000, seed=7), S.RANDOM_MESH_CAMERA, 64, 64, 8, 4, 4, None, {"stack_window": 1}),
             ("c5_plain", S.random_mesh(500_000, seed=7), S.RANDOM_MESH_CAMERA, 64, 64, 8, 4, 4, None, {"stack_window": 2}),
             ("c1_quant", scenes.cbox(), scenes.CBOX_CAM, w, h, depth, frames, att, g["seeds_in"], {"quantized": 1}),
             ("c5_window_quant", S.random_mesh(500_000, seed=7), S.RANDOM_MESH_CAMERA, 64, 64, 8, 4, 4, None,
              {"stack_window": 1, "quantized": 1})]
    for name, data, camj, w, h, depth, frames, att, seeds, tune in cases:
        for mode in (L.MODE_EXACT, L.MODE_NOPRUNE):
            for sched in (L.SCHED_SINGLE, L.SCHED_PAIRED):
                rnd.set_tuning(**tune)
                dsc = rnd.upload(data)
                st = rnd.new_state(w, h, seeds)
                rnd.render_frames(dsc, S.parse_camera(camj), st, depth, att, frames, mode=mode, schedule=sched,
                                  frames_per_launch=2)
                s = rnd.stats()
                out = {"case": name, "mode": mode, "schedule": sched, "violations": s["debug_violations"],
                       "stack_window": s["stack_window"], "digest": digest(st)}
                out["quantized"] = s["quantized"]
                if name.startswith("c1"):
                    out["golden"] = (st.hist.cpu().numpy().tobytes() == np.ascontiguousarray(g["hist"]).tobytes()
                                     and np.array_equal(st.count.cpu().numpy(), g["count"])
                                     and np.array_equal(st.seeds_np(), g["seeds"]))
                print(json.dumps(out), flush=True)
                dsc.close()
    rnd.set_tuning()


if __name__ == "__main__":
    main()
