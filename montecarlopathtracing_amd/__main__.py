"""Command line: render a reference config.json on the GPU(s) and write the .hdr,
or, for a "testbvh" / "testall" entry, print the BVH metrics (main.cpp:11-25).

    python -m montecarlopathtracing_amd [config.json] [--configid N] [--out DIR] [--preview PNG]
    torchrun --nproc-per-node 8 -m montecarlopathtracing_amd config.json   (row-stripe tiles)
"""
import argparse
import os
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser(prog="montecarlopathtracing_amd")
    ap.add_argument("config", nargs="?", default="config.json")
    ap.add_argument("--configid", type=int, default=None)
    ap.add_argument("--out", default=".")
    ap.add_argument("--frames", type=int, default=None, help="override attempt+1 frames")
    ap.add_argument("--preview", default=None, help="also write the gamma-2.2 display image (testkernel.cl) as PNG")
    a = ap.parse_args(argv)
    from . import config as C
    cfg = C.Config(a.config, a.configid)
    if cfg.TESTALL() or cfg.TESTBVH():
        from . import bvhtest
        bvhtest.run(cfg, root=os.path.dirname(os.path.abspath(a.config)))
        return 0
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        return _main_dist(a)
    from .app import App
    app = App(a.config, a.configid, out_dir=a.out)
    t0 = time.time()
    if a.frames:
        app.update(a.frames)
        path = app.output_picture()
    else:
        path = app.run()
    print("wrote %s (%dx%d, %d frames, %.2f s)" % (path, app.w, app.h, app.attempt_count, time.time() - t0))
    if a.preview:
        from . import scene as S
        print("wrote", S.write_png(a.preview, app.preview()))
    return 0


def _main_dist(a):
    import torch
    import torch.distributed as dist

    from . import config as C
    from . import dist as D
    from . import render as R
    from . import scene as S
    from .app import config_scene
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MCPT_DIST_SHARED_GPU=1 rehearses the N-rank job on a one-GPU box: every
    # rank on device 0, gloo for the one reduce (tests/test_gpu_dist.py)
    shared = os.environ.get("MCPT_DIST_SHARED_GPU") == "1"
    if shared:
        local = 0
    torch.cuda.set_device(local)
    if shared:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = C.Config(a.config, a.configid)
    if not cfg.USEOPENCL():
        raise ValueError('config has "opencl": false — the reference throws "Not Implemented" here')
    root = os.path.dirname(os.path.abspath(a.config))
    # the same scene and tree as App.init: the GPU treelet pass over a fresh
    # HLBVH for every bvhtype (scenebuild.cpp:66-95)
    data = config_scene(cfg, root, local)
    rnd = R.Renderer(local)
    sc = rnd.upload(data)
    w, h = cfg.WIDTH(), cfg.HEIGHT()
    frames = a.frames or cfg.MAXATTEPMT() + 1
    out = D.render_distributed(rnd, sc, S.parse_camera(cfg.GETCAMERA()), w, h, cfg.MAXDEPTH(), cfg.MAXATTEPMT(),
                               frames, R.default_seeds(w * h))
    if dist.get_rank() == 0:
        path = os.path.join(a.out, cfg.GETOBJNAME() + ".hdr")
        S.write_hdr(path, out[0].reshape(h, w, 4), flip=True)
        print("wrote", path)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
