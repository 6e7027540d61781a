"""Test helper: ctypes binding of the CPU oracle (oracle/liboracle.so).
Test infrastructure only — the product never loads this library."""
import ctypes
import os

import numpy as np

from montecarlopathtracing_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "oracle", "liboracle.so")
_so = None
P = L.ptr
i32, i64 = ctypes.c_int32, ctypes.c_int64


def available():
    return os.path.exists(PATH)


def so():
    global _so
    if _so is None:
        _so = ctypes.CDLL(PATH)
        _so.oracle_encode_hdr.restype = ctypes.c_int64
        _so.oracle_bvh_sah.restype = ctypes.c_float
        _so.oracle_bvh_lcv.restype = ctypes.c_float
    return _so


def parse_camera(cj):
    out = np.zeros(1, L.CAMERA)
    a = [np.asarray(cj[k], np.float64) for k in ("position", "lookat", "up")]
    so().oracle_parse_camera(P(a[0]), P(a[1]), P(a[2]), ctypes.c_double(cj["fov"]), P(out))
    return out


def pack_triangles(tris, idx):
    t = tris.copy()
    so().oracle_pack_triangles(P(t), P(np.ascontiguousarray(idx, np.int32)), i64(len(t)))
    return t


def build_hlbvh(tris):
    nodes = np.zeros(2 * len(tris) - 1, L.BVHNODE)
    so().oracle_build_hlbvh(P(np.ascontiguousarray(tris)), i64(len(tris)), P(nodes))
    return nodes


def generate(cam, w, h):
    rays = np.zeros(w * h, L.RAY)
    so().oracle_generate(P(cam), i32(w), i32(h), P(rays))
    return rays


def intersect(data, rays, hits=None, tmin=0.001):
    hits = np.zeros(len(rays), L.HIT) if hits is None else hits.copy()
    so().oracle_intersect(P(data.tris), P(data.nodes), P(np.ascontiguousarray(rays)), i64(len(rays)), P(hits),
                          ctypes.c_float(tmin))
    return hits


def shade(data, rays, hits, colors, seeds, max_depth):
    rays, colors, seeds = rays.copy(), colors.copy(), seeds.copy()
    so().oracle_shade(P(data.mats), P(rays), P(np.ascontiguousarray(hits)), P(colors), P(seeds), i64(len(rays)),
                      i32(max_depth))
    return rays, colors, seeds


def accumulate(colors, hist, count, max_attempt):
    colors, hist, count = colors.copy(), hist.copy(), count.copy()
    so().oracle_accumulate(P(colors), P(hist), P(count), i64(len(count)), i32(max_attempt))
    return colors, hist, count


def render(data, cam, w, h, max_depth, frames, max_attempt, seeds, frame_begin=0, threads=0, pixels=None,
           hist=None, count=None, prune=False):
    seeds = np.ascontiguousarray(seeds, np.uint32).copy()
    hist = np.zeros((w * h, 4), np.float32) if hist is None else hist.copy()
    count = np.zeros(w * h, np.int32) if count is None else count.copy()
    stats = np.zeros(4, np.uint64)
    so().oracle_set_prune(int(prune))
    if pixels is None:
        so().oracle_render(P(cam), P(data.tris), P(data.nodes), P(data.mats), i32(w), i32(h), i32(max_depth),
                           i32(frame_begin), i32(frames), i32(max_attempt), P(seeds), P(hist), P(count), i32(threads),
                           P(stats))
    else:
        px = np.ascontiguousarray(pixels, np.int32)
        so().oracle_render_pixels(P(cam), P(data.tris), P(data.nodes), P(data.mats), i32(w), i32(h), P(px),
                                  i64(len(px)), i32(max_depth), i32(frame_begin), i32(frames), i32(max_attempt),
                                  P(seeds), P(hist), P(count), i32(threads), P(stats))
    so().oracle_set_prune(0)
    return hist, count, seeds, stats


def encode_hdr(rgba, flip=True):
    a = np.ascontiguousarray(rgba, np.float32)
    h, w = a.shape[:2]
    n = so().oracle_encode_hdr(i32(w), i32(h), P(a), i32(int(flip)), None, i64(0))
    buf = np.zeros(n, np.uint8)
    so().oracle_encode_hdr(i32(w), i32(h), P(a), i32(int(flip)), P(buf), i64(n))
    return buf.tobytes()


def treelet(nodes):
    """TreeletBVH<CPU> restated (oracle/mcpt_oracle_treelet.cpp): (status, nodes)."""
    out = np.ascontiguousarray(nodes).copy()
    rc = so().oracle_treelet(P(out), i64(len(out)))
    return rc, out


def treelet_gpu(nodes, rcp_bits=0, options=0):
    """TreeletBVH<GPU> (treeletBVH.cl) restated (oracle/mcpt_oracle_treelet_gpu.cpp):
    (status, nodes, stats[8]).  rcp_bits: the GPU's v_rcp_f32(frexp_mant(rootArea))
    as uint32 bits (0 = correctly rounded); options: bit 0 lowest-lane stores,
    bit 1 refit divided by rootArea (sensitivity knobs, not the kernel)."""
    out = np.ascontiguousarray(nodes).copy()
    stats = np.zeros(8, np.int64)
    rc = so().oracle_treelet_gpu(P(out), i64(len(out)), ctypes.c_uint32(int(rcp_bits)), i32(options), P(stats))
    return rc, out, stats


def root_area_mant(nodes):
    """frexp mantissa of treeletBVH.cl's rootArea (AREA(nodes[0]), :245): the
    float whose v_rcp_f32 the GPU tests feed to treelet_gpu()."""
    so().oracle_treelet_gpu_root_mant.restype = ctypes.c_float
    return np.float32(so().oracle_treelet_gpu_root_mant(P(np.ascontiguousarray(nodes[:1]))))


def bvh_sah(nodes):
    return so().oracle_bvh_sah(P(np.ascontiguousarray(nodes)), i64(len(nodes)))


def bvh_lcv(nodes, cam, w, h):
    """(LCV, per-ray leaf counts indexed i*h + j)."""
    counts = np.zeros(w * h, np.uint32)
    v = so().oracle_bvh_lcv(P(np.ascontiguousarray(nodes)), i64(len(nodes)), P(cam), i32(w), i32(h), P(counts))
    return v, counts


def bvh_epo(nodes, tris):
    """Per-triangle (EPO area, triangle area) of EPO.cl, CPU restatement."""
    n = len(tris)
    e, a = np.zeros(n, np.float32), np.zeros(n, np.float32)
    so().oracle_bvh_epo(P(np.ascontiguousarray(nodes)), P(np.ascontiguousarray(tris)), i64(n), P(e), P(a))
    return e, a
