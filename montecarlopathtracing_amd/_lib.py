"""ctypes binding of libmcpt_hip.so (the C ABI declared in include/mcpt_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
montecarlopathtracing_amd/csrc``) into ``montecarlopathtracing_amd/lib/``.
There is no fallback: if the shared object is missing or does not export the
ABI, :func:`lib` raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCPT_LIB_OVERRIDE") or os.path.join(_HERE, "lib", "libmcpt_hip.so")  # override: tuning sweeps only

# ------------------------------------------------ record dtypes (objdef.h)
CAMERA = np.dtype([("center", "<f4", 4), ("direction", "<f4", 4), ("up", "<f4", 4),
                   ("horizontal", "<f4", 4), ("arg", "<f4"), ("tmin", "<f4"),
                   ("camera_type", "<u4"), ("pad", "<f4")])
RAY = np.dtype([("origin", "<f4", 4), ("direction", "<f4", 4), ("ratio", "<f4", 4)])
HIT = np.dtype([("normal", "<f4", 4), ("point", "<f4", 4), ("t", "<f4"),
                ("triangle_id", "<u4"), ("material_id", "<u4"), ("pad", "<u4")])
TRIANGLE = np.dtype([("v", "<f4", (3, 4)), ("normal", "<f4", 4)])
MATERIAL = np.dtype([("type", "<i4"), ("Ni", "<f4"), ("Ns", "<f4"), ("pad", "<f4"),
                     ("kd", "<f4", 4), ("ka_ks", "<f4", 4)])
BVHNODE = np.dtype([("bbmin", "<f4", 4), ("bbmax", "<f4", 4), ("pad", "<f4", 4),
                    ("parent", "<i4"), ("left", "<i4"), ("right", "<i4"), ("pad2", "<i4")])
for _dt, _sz in ((CAMERA, 80), (RAY, 48), (HIT, 48), (TRIANGLE, 64), (MATERIAL, 48), (BVHNODE, 64)):
    assert _dt.itemsize == _sz

ABI_VERSION = 4  # include/mcpt_hip.h MCPT_ABI_VERSION
MCPT_DIFFUSE, MCPT_GLOSSY, MCPT_TRANSPARENT, MCPT_LIGHT = 1, 2, 3, 4
MODE_EXACT, MODE_NOPRUNE = 0, 1
SCHED_SINGLE, SCHED_PAIRED = 0, 1  # mcpt_render_params.schedule
TERMINATED = 0xFF000000


class RenderParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "width", "height", "max_depth", "max_attempt", "frame_begin", "frames", "stripe_rows",
        "stripe_index", "stripe_count", "mode", "frames_per_launch", "schedule")]


class Stats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("node_visits", ctypes.c_uint64),
                ("tri_tests", ctypes.c_uint64), ("bad_material", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double), ("launches", ctypes.c_int32), ("frames_per_block", ctypes.c_int32),
                ("wave_node_phases", ctypes.c_uint64), ("wave_leaf_phases", ctypes.c_uint64),
                ("wave_shade_phases", ctypes.c_uint64), ("order_fallbacks", ctypes.c_uint64),
                ("wave_iterations", ctypes.c_uint64), ("lane_waiting", ctypes.c_uint64), ("lane_idle", ctypes.c_uint64),
                ("stack_window", ctypes.c_int32), ("workgroups", ctypes.c_int32),
                ("debug_violations", ctypes.c_uint64), ("phase_ticks", ctypes.c_uint64 * 4),
                ("leaf_rejects", ctypes.c_uint64), ("quantized", ctypes.c_int32), ("primary_cache", ctypes.c_int32),
                ("primary_ms", ctypes.c_double), ("top_levels", ctypes.c_int32)]


class Tuning(ctypes.Structure):
    """mcpt_tuning: launch-plan knobs of k_render (speed only; 0 = default)."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "leaf_threshold", "shade_threshold", "queue_chunk", "block_entries", "max_block_frames", "stack_window",
        "lds_pad", "queues", "fetch_threshold", "quantized", "primary_cache", "last_block_frames", "tile_order", "pixel_spread",
        "top_levels")]


class MCPTError(RuntimeError):
    """A C-ABI call returned a negative status."""


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F32 = ctypes.c_float
_D = ctypes.c_double
_S = ctypes.c_char_p

# name -> (restype, argtypes); every symbol include/mcpt_hip.h declares
SIGNATURES = {
    "mcpt_abi_version": (_I32, []),
    "mcpt_version": (_S, []),
    "mcpt_last_error": (_S, []),
    "mcpt_parse_camera": (_I32, [_P, _P, _P, _D, _P]),
    "mcpt_classify_material": (_I32, [_F32, _P, _P, _P, _F32, _P]),
    "mcpt_load_obj": (_I32, [_S, _S, _P, _P, _P, _P, _P]),
    "mcpt_pack_triangles": (_I32, [_P, _P, _I64]),
    "mcpt_build_hlbvh": (_I32, [_P, _I64, _P]),
    "mcpt_bvh_stack_depth": (_I32, [_P, _I64, _P]),
    "mcpt_write_hdr": (_I32, [_S, _I32, _I32, _P, _I32]),
    "mcpt_encode_hdr": (_I64, [_I32, _I32, _P, _I32, _P, _I64]),
    "mcpt_ctx_create": (_I32, [_I32, _P]),
    "mcpt_ctx_destroy": (_I32, [_P]),
    "mcpt_device_count": (_I32, [_P]),
    "mcpt_scene_upload": (_I32, [_P, _P, _I64, _P, _I64, _P, _I32, _P]),
    "mcpt_scene_destroy": (_I32, [_P]),
    "mcpt_scene_upload_device": (_I32, [_P, _P, _I64, _P, _I64, _P, _I32, _P, _P]),
    "mcpt_scene_read": (_I32, [_P, _I32, _P, _I64, _P]),
    "mcpt_render_frames": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "mcpt_generate_rays": (_I32, [_P, _P, _I32, _I32, _P, _P]),
    "mcpt_intersect": (_I32, [_P, _P, _P, _I64, _P, _F32, _I32, _P]),
    "mcpt_shade": (_I32, [_P, _P, _P, _P, _P, _P, _I64, _I32, _P]),
    "mcpt_accumulate": (_I32, [_P, _P, _P, _P, _I64, _I32, _P]),
    "mcpt_gamma_preview": (_I32, [_P, _P, _P, _I64, _P]),
    "mcpt_set_tuning": (_I32, [_P, _P]),
    "mcpt_get_tuning": (_I32, [_P, _P]),
    "mcpt_drop_caches": (_I32, [_P]),
    "mcpt_state_create": (_I32, [_P, _I32, _I32, _P, _P]),
    "mcpt_state_buffers": (_I32, [_P, _P, _P, _P]),
    "mcpt_download": (_I32, [_P, _P, _P, _P, _P, _P]),
    "mcpt_upload": (_I32, [_P, _P, _P, _P, _P, _P]),
    "mcpt_state_destroy": (_I32, [_P]),
    "mcpt_set_stats": (_I32, [_P, _I32]),
    "mcpt_get_stats": (_I32, [_P, _P]),
    "mcpt_get_wave_log": (_I32, [_P, _P, _I64, _P]),
    "mcpt_set_pixel_segments": (_I32, [_P, _P, _P, _I64]),
    "mcpt_get_primary_cost": (_I32, [_P, _P, _I64, _P]),
    "mcpt_get_entry_log": (_I32, [_P, _P, _I64, _P, _P]),
    "mcpt_selfcheck_trig": (_I32, [_P, _P, _P]),
    "mcpt_selfcheck_pow": (_I32, [_P, _P, _I32, _P]),
    "mcpt_measure_read_bw": (_I32, [_P, _I64, _P]),
    "mcpt_gather_probe": (_I32, [_P, _I32, _I64, _P]),
    "mcpt_build_hlbvh_device": (_I32, [_P, _I64, _P, _P]),
    "mcpt_treelet_device": (_I32, [_P, _I64, _P]),
    "mcpt_treelet_gpu_device": (_I32, [_P, _I64, _P]),
    "mcpt_treelet_gpu": (_I32, [_P, _I64]),
    "mcpt_bvh_sah": (_I32, [_P, _I64, _P]),
    "mcpt_bvh_epo_device": (_I32, [_P, _P, _I64, _P, _P, _P, _P, _P]),
    "mcpt_bvh_lcv_device": (_I32, [_P, _I64, _P, _I32, _I32, _P, _P, _P]),
}

_lib = None


def lib():
    """Load libmcpt_hip.so (once) and declare every ABI function."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MCPTError("libmcpt_hip.so not built: run __graft_entry__.build() "
                            "or make -C montecarlopathtracing_amd/csrc (%s missing)" % LIB_PATH)
        # torch ships its own HIP runtime; the library must bind to that same
        # instance (device tensors cross the ABI), so torch is loaded first.
        # Loading the library first makes torch reuse /opt/rocm's runtime by
        # soname and leaves one of the two without a device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        so = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("MCPT_LIB_OVERRIDE") and not hasattr(so, name):
                continue  # an older build under A/B timing (tools/ab.py) may lack newer entry points
            fn = getattr(so, name)
            fn.restype = res
            fn.argtypes = args
        if hasattr(so, "mcpt_abi_version") and so.mcpt_abi_version() != ABI_VERSION:
            raise MCPTError("libmcpt_hip.so implements ABI %d, this binding ABI %d (rebuild one of them)" % (
                so.mcpt_abi_version(), ABI_VERSION))
        _lib = so
    return _lib


def check(rc):
    """Raise MCPTError with the library's message for a negative status."""
    if rc < 0:
        msg = lib().mcpt_last_error()
        raise MCPTError("mcpt error %d: %s" % (rc, msg.decode() if msg else ""))
    return rc


def ptr(a):
    """Pointer of a numpy array (host) or a torch tensor (device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(a.data_ptr())
