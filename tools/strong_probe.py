"""One rank's share of a strong-scaled C4 (1920x1080 striped over N ranks),
timed on one GPU for several frames-per-block values."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from montecarlopathtracing_amd import _lib as L  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import oracle as O  # noqa: E402,F401  (scenes import path)
from tests import scenes  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    data = scenes.dining()
    data = data.with_nodes(R.treelet_device(data.nodes))
    cam = S.parse_camera(scenes.DINING_CAM)
    r = R.Renderer(0)
    dsc = r.upload(data)
    dsc.schedule = L.SCHED_PAIRED
    w, h = 1920, 1080
    for fpl in (16, 8, 4, 2):
        st = r.new_state(w, h)
        kw = dict(stripe_rows=16, stripe_index=0, stripe_count=n, frames_per_launch=fpl)
        r.render_frames(dsc, cam, st, 16, 1 << 20, frames, **kw)
        ms = []
        for _ in range(3):
            r.render_frames(dsc, cam, st, 16, 1 << 20, frames, **kw)
            torch.cuda.synchronize()
            ms.append(r.stats()["kernel_ms"])
        rows = sum(min(16, max(0, h - (s * n) * 16)) for s in range((h + 16 * n - 1) // (16 * n)))
        print("N=%d fpl=%d frames=%d: %.3f ms (min of 3), %.0f Msamples/s for this rank's %d rows" % (
            n, fpl, frames, min(ms), w * rows * frames * 16 / min(ms) / 1e3, rows))


if __name__ == "__main__":
    main()
