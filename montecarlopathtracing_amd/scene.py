"""Scene-side host pipeline: the reference's ThirdPartyWrapper::loadObject,
Auxiliary::parseCamera, SceneCL packing and HLBVH<CPU> build, all running in
the native host half of libmcpt_hip.so (csrc/mcpt_host.cpp).

    load_object   MCPT/thirdpartywrapper.cpp:25-99
    parse_camera  MCPT/auxiliary.cpp:20-71
    pack_triangles MCPT/scenebuild.cpp:58-62
    build_hlbvh   MCPT/BVH/hlbvh.cpp:92-200
"""
import ctypes

import numpy as np

from . import _lib as L


def load_object(directory, objname):
    """OBJ + MTL -> (triangles[TRIANGLE], materials[MATERIAL], mat_index[int32])."""
    lib = L.lib()
    nt, nm = ctypes.c_int64(0), ctypes.c_int32(0)
    d, o = directory.encode(), objname.encode()
    L.check(lib.mcpt_load_obj(d, o, None, None, ctypes.byref(nt), None, ctypes.byref(nm)))
    tris = np.zeros(nt.value, L.TRIANGLE)
    idx = np.zeros(nt.value, np.int32)
    mats = np.zeros(max(nm.value, 0), L.MATERIAL)
    L.check(lib.mcpt_load_obj(d, o, L.ptr(tris), L.ptr(idx), ctypes.byref(nt), L.ptr(mats), ctypes.byref(nm)))
    return tris, mats, idx


def classify_material(ior=1.0, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0), shininess=1.0):
    """One MTL record -> Material (thirdpartywrapper.cpp:65-97)."""
    out = np.zeros(1, L.MATERIAL)
    a = np.asarray(ambient, np.float32)
    dfs = np.asarray(diffuse, np.float32)
    s = np.asarray(specular, np.float32)
    L.check(L.lib().mcpt_classify_material(float(ior), L.ptr(a), L.ptr(dfs), L.ptr(s), float(shininess), L.ptr(out)))
    return out[0]


def parse_camera(camera_json):
    """JSON camera object (position/lookat/up/fov) -> Camera record."""
    pos = np.asarray(camera_json["position"], np.float64)
    look = np.asarray(camera_json["lookat"], np.float64)
    up = np.asarray(camera_json["up"], np.float64)
    out = np.zeros(1, L.CAMERA)
    L.check(L.lib().mcpt_parse_camera(L.ptr(pos), L.ptr(look), L.ptr(up), float(camera_json["fov"]), L.ptr(out)))
    return out


def pack_triangles(tris, mat_index):
    """normal = normalize(cross(v1-v0, v2-v0)), normal.w <- material index bits (copy)."""
    t = np.ascontiguousarray(tris.copy())
    m = np.ascontiguousarray(np.asarray(mat_index, np.int32))
    if len(m) != len(t):
        raise ValueError("one material index per triangle")
    L.check(L.lib().mcpt_pack_triangles(L.ptr(t), L.ptr(m), len(t)))
    return t


def build_hlbvh(tris):
    """HLBVH<CPU>: 2n-1 BVHNode records (root 0, leaves at [n-1, 2n-2])."""
    n = len(tris)
    if n == 0:
        raise ValueError("empty scene")
    nodes = np.zeros(2 * n - 1, L.BVHNODE)
    t = np.ascontiguousarray(tris)
    L.check(L.lib().mcpt_build_hlbvh(L.ptr(t), n, L.ptr(nodes)))
    return nodes


def bvh_stack_depth(nodes):
    d = ctypes.c_int32(0)
    L.check(L.lib().mcpt_bvh_stack_depth(L.ptr(np.ascontiguousarray(nodes)), len(nodes), ctypes.byref(d)))
    return d.value


def encode_hdr(rgba, flip=True):
    """RGBE bytes exactly as stbi_write_hdr writes them (outputPicture flips)."""
    a = np.ascontiguousarray(rgba, np.float32)
    h, w = a.shape[0], a.shape[1]
    n = L.check(L.lib().mcpt_encode_hdr(w, h, L.ptr(a), int(flip), None, 0))
    buf = np.zeros(n, np.uint8)
    L.check(L.lib().mcpt_encode_hdr(w, h, L.ptr(a), int(flip), L.ptr(buf), n))
    return buf.tobytes()


def write_hdr(path, rgba, flip=True):
    """ThirdPartyWrapper::outputPicture (thirdpartywrapper.cpp:14-23)."""
    a = np.ascontiguousarray(rgba, np.float32)
    L.check(L.lib().mcpt_write_hdr(path.encode(), a.shape[1], a.shape[0], L.ptr(a), int(flip)))


def preview_rgb8(preview, flip=True):
    """8-bit RGB of a gamma-encoded preview (mcpt_gamma_preview's float4s):
    round(clamp(c, 0, 1) * 255) per channel; flip=True puts the image's top
    row first, as the .hdr dump does (row 0 of the render is its bottom)."""
    a = np.asarray(preview, np.float32)[..., :3]
    a = np.nan_to_num(a, nan=0.0, posinf=1.0, neginf=0.0)
    q = np.floor(np.clip(a, 0.0, 1.0) * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)
    return np.ascontiguousarray(q[::-1] if flip else q)


def write_png(path, preview, flip=True):
    """The display's gamma-2.2 image as a PNG (the optional
    preview of testkernel.cl's pass): 8-bit RGB, no interlace, zlib-compressed
    rows with filter 0."""
    import struct
    import zlib
    q = preview_rgb8(preview, flip)
    h, w = q.shape[:2]
    raw = b"".join(b"\x00" + q[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
           + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
    with open(path, "wb") as fh:
        fh.write(png)
    return path


class SceneData:
    """Host-side scene: packed triangles, HLBVH nodes, materials."""

    def __init__(self, tris, nodes, mats):
        self.tris, self.nodes, self.mats = tris, nodes, mats

    def with_nodes(self, nodes):
        """Same triangles and materials over another BVH (e.g. a treelet pass)."""
        return SceneData(self.tris, nodes, self.mats)

    @classmethod
    def from_obj(cls, directory, objname, material_override=None):
        tris, mats, idx = load_object(directory, objname)
        if (idx < 0).any():
            raise ValueError("face without a known material")
        if material_override is not None:
            mats = material_override(mats)
        packed = pack_triangles(tris, idx)
        return cls(packed, build_hlbvh(packed), mats)

    @classmethod
    def from_arrays(cls, verts, mat_index, mats, build=None):
        """verts: (n, 3, 3) float32 triangle corners.  `build` makes the
        HLBVH from the packed triangles (default: the host build_hlbvh;
        render.build_hlbvh_host_nodes builds the same tree on the GPU)."""
        v = np.asarray(verts, np.float32)
        t = np.zeros(len(v), L.TRIANGLE)
        t["v"][:, :, :3] = v
        packed = pack_triangles(t, mat_index)
        return cls(packed, (build or build_hlbvh)(packed), mats)


def diffuse_only(mats):
    """C2's material override (BASELINE.json configs[1]): every non-light
    material becomes DIFFUSE with its kd (already Kd/pi); glass has Kd = 0."""
    m = mats.copy()
    for i in range(len(m)):
        if m[i]["type"] != L.MCPT_LIGHT:
            m[i]["type"] = L.MCPT_DIFFUSE
    return m


# ------------------------------------------------------------- synthetic scenes
RANDOM_MESH_CAMERA = {"position": [50.0, 50.0, -150.0], "lookat": [50.0, 50.0, 50.0], "up": [0, 1, 0], "fov": 45.0}


def random_mesh(n, seed=42, extent=100.0, build=None):
    """BASELINE.json configs[4] / SURVEY.md §8(d) C5: n random triangles,
    centres uniform in [0, extent]^3, corners = centre + U[-h, h]^3 with
    h = 0.5 * extent / n^(1/3); diffuse 0.5; one emissive quad (Ka 10)
    above the volume.  numpy PCG64(seed) stands in for the survey's PCG32."""
    rng = np.random.Generator(np.random.PCG64(seed))
    h = 0.5 * extent / float(n) ** (1.0 / 3.0)
    c = rng.uniform(0.0, extent, (n, 1, 3)).astype(np.float32)
    v = (c + rng.uniform(-h, h, (n, 3, 3)).astype(np.float32)).astype(np.float32)
    y = np.float32(1.2 * extent)
    lo, hi = np.float32(0.25 * extent), np.float32(0.75 * extent)
    quad = np.array([[[lo, y, lo], [hi, y, lo], [hi, y, hi]], [[lo, y, lo], [hi, y, hi], [lo, y, hi]]], np.float32)
    verts = np.concatenate([v, quad], axis=0)
    mat_index = np.zeros(len(verts), np.int32)
    mat_index[-2:] = 1
    mats = np.zeros(2, L.MATERIAL)
    mats[0] = classify_material(1.0, (0, 0, 0), (0.5, 0.5, 0.5), (0, 0, 0), 1.0)
    mats[1] = classify_material(1.0, (10, 10, 10), (0, 0, 0), (0, 0, 0), 1.0)
    return SceneData.from_arrays(verts, mat_index, mats, build=build)
