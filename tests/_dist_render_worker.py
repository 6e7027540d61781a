"""One rank of tests/test_gpu_dist.py: dist.render_distributed over a gloo
group whose ranks share the box's one GPU, or over RCCL ("nccl") with one rank
(RCCL refuses two ranks on one device); rank 0 saves the reduced image.

    _dist_render_worker.py <out.npz> [gloo|nccl]"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from montecarlopathtracing_amd import dist as D  # noqa: E402
from montecarlopathtracing_amd import render as R  # noqa: E402
from montecarlopathtracing_amd import scene as S  # noqa: E402
from tests import scenes  # noqa: E402

W, H, DEPTH, FRAMES = 160, 120, 6, 4


def main(out, backend):
    torch.cuda.set_device(0)
    dist.init_process_group(backend)
    rnd = R.Renderer(0)
    sc = rnd.upload(scenes.cbox())
    res = D.render_distributed(rnd, sc, S.parse_camera(scenes.CBOX_CAM), W, H, DEPTH, 1 << 20, FRAMES,
                               R.default_seeds(W * H), stripe_rows=16)
    if dist.get_rank() == 0:
        np.savez(out, hist=res[0], count=res[1], seeds=res[2])
    sc.close()
    rnd.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "gloo")
