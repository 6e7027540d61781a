"""__graft_entry__.smoke(): one small invocation of the hot path on cuda:0,
checked against the CPU oracle on the same seeded input."""
import os

import numpy as np


def run():
    import torch

    from montecarlopathtracing_amd import _lib as L
    from montecarlopathtracing_amd import render as R
    from montecarlopathtracing_amd import scene as S

    from . import oracle as O
    from . import scenes

    assert torch.cuda.is_available(), "smoke needs a GPU"
    w = h = 64
    depth, frames, att = 4, 4, 4
    data, cam = scenes.cbox(), S.parse_camera(scenes.CBOX_CAM)
    seeds = R.default_seeds(w * h)
    rnd = R.Renderer(0)
    dsc = rnd.upload(data)
    st = rnd.new_state(w, h, seeds)
    rnd.render_frames(dsc, cam, st, depth, att, frames)
    torch.cuda.synchronize()
    mine = st.hist.cpu().numpy()
    oh, oc, _, _ = O.render(data, cam, w, h, depth, frames, att, seeds)
    close = (np.abs(mine - oh) <= 1e-5 * np.maximum(np.abs(oh), 1e-3)).all(axis=1).mean()
    same_count = (st.count.cpu().numpy() == oc).mean()
    assert close >= 0.95 and same_count >= 0.95, (close, same_count)
    assert os.path.samefile(os.path.dirname(L.LIB_PATH), os.path.join(scenes.ROOT, "montecarlopathtracing_amd", "lib"))
    print("smoke ok: %.4f pixels within 1e-5, %.4f counts equal, mean %s" % (close, same_count, mine[:, :3].mean(0)))
    dsc.close()
    rnd.close()
