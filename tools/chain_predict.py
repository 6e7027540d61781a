"""How well the primary-ray cost (the only per-pixel cost known before a call's
frames run) finds the long per-pixel chains: reads the per-pixel arrays
tools/chain_probe.py saves (gpurun_out/chain_<workload>.npy: segments, busy
loop iterations, primary cost) and prints, for chains above a few lengths,
how many fall among the k pixels / tiles with the dearest primary ray.

    python tools/chain_predict.py gpurun_out/chain_C2.npy --width 1024
"""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npy")
    ap.add_argument("--width", type=int, default=1024)
    a = ap.parse_args()
    c, it, pc = np.load(a.npy).astype(np.int64)
    w = a.width
    h = len(it) // w
    print("pixels %d, chain iterations mean %.1f p50 %d p99 %d max %d; corr(primary cost, iterations) %.3f"
          % (len(it), it.mean(), np.percentile(it, 50), np.percentile(it, 99), it.max(), np.corrcoef(pc, it)[0, 1]))
    order = np.argsort(-pc, kind="stable")
    for thr in (2500, 3000, 3500):
        hot = np.where(it > thr)[0]
        row = ["chains > %d: %d;" % (thr, len(hot))]
        for k in (1024, 2048, 4096, 8192, 16384):
            row.append("%d in the dearest %d" % (np.isin(hot, order[:k]).sum(), k))
        print(" ".join(row))
    if h % 8 == 0 and w % 8 == 0:
        tiles_max = pc.reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64).max(1)
        hot = np.where(it > 3000)[0]
        hot_tiles = np.unique((hot // w // 8) * (w // 8) + (hot % w) // 8)
        tord = np.argsort(-tiles_max, kind="stable")
        print("tiles holding a chain > 3000: %d; " % len(hot_tiles)
              + ", ".join("%d among the dearest %d" % (np.isin(hot_tiles, tord[:k]).sum(), k) for k in (16, 64, 256)))


if __name__ == "__main__":
    main()
