"""Test helper: the reference's own OpenCL kernels on the GPU (oracle/_ref).

Loads oracle/_ref/libref_runner.so, which launches the unmodified reference
kernels compiled for gfx950 (oracle/Makefile).  Test infrastructure only.
"""
import ctypes
import os

import numpy as np

from montecarlopathtracing_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
_so = None


def available():
    return os.path.exists(os.path.join(REF_DIR, "libref_runner.so")) and \
        os.path.exists(os.path.join(REF_DIR, "intersect.co"))


def so():
    global _so
    if _so is None:
        s = ctypes.CDLL(os.path.join(REF_DIR, "libref_runner.so"))
        s.ref_last_error.restype = ctypes.c_char_p
        for n in ("ref_init", "ref_generate", "ref_intersect", "ref_shade", "ref_accumulate", "ref_render", "ref_epo",
                  "ref_rcp_f32"):
            getattr(s, n).restype = ctypes.c_int
        if s.ref_init(REF_DIR.encode()) != 0:
            raise RuntimeError(s.ref_last_error().decode())
        _so = s
    return _so


def _ck(rc):
    if rc != 0:
        raise RuntimeError("reference runner: " + so().ref_last_error().decode())


P = L.ptr
i64 = ctypes.c_int64
i32 = ctypes.c_int32


def generate(cam, w, h):
    rays = np.zeros(w * h, L.RAY)
    _ck(so().ref_generate(P(cam), i32(w), i32(h), P(rays)))
    return rays


def intersect(data, rays, tmin=0.001, hits=None):
    if hits is None:
        hits = np.zeros(len(rays), L.HIT)
    hits = hits.copy()
    _ck(so().ref_intersect(P(data.tris), i64(len(data.tris)), P(data.nodes), i64(len(data.nodes)), P(rays),
                           i64(len(rays)), P(hits), ctypes.c_float(tmin)))
    return hits


def shade(data, rays, hits, colors, seeds, max_depth):
    rays, colors, seeds = rays.copy(), colors.copy(), seeds.copy()
    _ck(so().ref_shade(P(data.mats), i32(len(data.mats)), P(rays), P(hits), P(colors), P(seeds), i64(len(rays)),
                       i32(max_depth)))
    return rays, colors, seeds


def accumulate(colors, hist, count, w, h, max_attempt):
    colors, hist, count = colors.copy(), hist.copy(), count.copy()
    _ck(so().ref_accumulate(P(colors), P(hist), P(count), i32(w), i32(h), i32(max_attempt)))
    return colors, hist, count


def render(data, cam, w, h, max_depth, frames, max_attempt, seeds):
    seeds = np.ascontiguousarray(seeds, np.uint32).copy()
    hist = np.zeros((w * h, 4), np.float32)
    count = np.zeros(w * h, np.int32)
    _ck(so().ref_render(P(cam), P(data.tris), i64(len(data.tris)), P(data.nodes), i64(len(data.nodes)),
                        P(data.mats), i32(len(data.mats)), i32(w), i32(h), i32(max_depth), i32(frames),
                        i32(max_attempt), P(seeds), P(hist), P(count)))
    return hist, count, seeds


def epo(nodes, tris):
    """EPO.cl calculateEPO (the reference's EPO_GPU kernel): per-triangle
    (EPO area, triangle area)."""
    n = len(tris)
    e, a = np.zeros(n, np.float32), np.zeros(n, np.float32)
    _ck(so().ref_epo(P(np.ascontiguousarray(nodes)), i64(len(nodes)), P(np.ascontiguousarray(tris)), i64(n), P(e),
                     P(a)))
    return e, a


def rcp_f32(x):
    """The GPU's v_rcp_f32 of each float (the hardware reciprocal the
    treeletBVH.cl restatement's 2.5-ulp division uses)."""
    a = np.ascontiguousarray(np.atleast_1d(x), np.float32).copy()
    out = np.zeros_like(a)
    _ck(so().ref_rcp_f32(P(a), P(out), i64(len(a))))
    return out

