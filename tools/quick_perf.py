"""Quick single-GPU timing of the fused path on the C2 configuration."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import scenes  # noqa: E402


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    w = h = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    depth = 8
    which = sys.argv[3] if len(sys.argv) > 3 else "cbox_diffuse"
    data = getattr(scenes, which)()
    camj = scenes.MIS_CAM if which == "mis" else scenes.CBOX_CAM
    cam = S.parse_camera(camj)
    r = R.Renderer(0)
    dsc = r.upload(data)
    for mode in (L.MODE_EXACT,):
        for stats in (True, False):
            r.set_stats(stats)
            st = r.new_state(w, h)
            r.render_frames(dsc, cam, st, depth, 1 << 20, 1, mode=mode)  # warm
            torch.cuda.synchronize()
            reps = 1 if stats else int(os.environ.get("QP_REPS", "7"))
            kms = []
            for _ in range(reps):  # median of reps launches (single launches vary by ~5 %)
                t0 = time.time()
                r.render_frames(dsc, cam, st, depth, 1 << 20, frames, mode=mode,
                                frames_per_launch=int(os.environ.get("QP_FPL", "0")))
                torch.cuda.synchronize()
                dt = time.time() - t0
                s = r.stats()
                kms.append(s["kernel_ms"])
            km = sorted(kms)[len(kms) // 2]
            nominal = w * h * frames * depth / (km / 1e3) / 1e6
            print("mode=%d stats=%d frames=%d nominal %.1f Msamples/s kernel_ms median %.2f (min %.2f max %.2f, %d reps)"
                  % (mode, stats, frames, nominal, km, min(kms), max(kms), reps))
            if stats:
                seg = s["segments"]
                print("   segments %.3g (%.2f/path) nodes/seg %.2f tris/seg %.2f bad %d order fallbacks %d "
                      "active Mseg/s %.1f" % (seg, seg / (w * h * frames), s["node_visits"] / seg,
                                              s["tri_tests"] / seg, s["bad_material"], s["order_fallbacks"],
                                              seg / dt / 1e6))
                if s["wave_node_phases"]:
                    print("   SIMT: node %.3f leaf %.3f shade %.3f (lanes active per phase / 64)" % (
                        s["node_visits"] / (64.0 * s["wave_node_phases"]),
                        s["tri_tests"] / (64.0 * max(s["wave_leaf_phases"], 1)),
                        seg / (64.0 * max(s["wave_shade_phases"], 1))))


if __name__ == "__main__":
    main()
