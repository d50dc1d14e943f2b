"""ctypes binding of libprt (include/prt.h) — the only way the product reaches the GPU.

There is no CPU fallback: if libprt.so is missing or a call fails, a
PrtError is raised with the library's message.
"""
import ctypes
import os

import numpy as np

from .build import LIB

ABI_VERSION = 4        # include/prt.h PRT_ABI_VERSION
PRT_OK = 0
PRT_ERR_UNSUP = -5      # feature not supported by this build
PRT_ERR_INTERNAL = -6   # device-side check failed (traversal watchdog)
PRT_FLAG_STATS = 0x1
PRT_FLAG_TIME = 0x2
PRT_FLAG_NO_PRIMARY_KERNEL = 0x4   # rejected (PRT_ERR_UNSUP) since round 4: camera rays come from the camera kernel
PRT_FLAG_MIS_NEE = 0x8
# trace-kernel variant ids 1..VAR_LAST of the reference estimator (pyrenderer_amd/csrc/prt_kernels.h
# kVar*); the MIS direct-lighting estimator's variants (PRT_FLAG_MIS_NEE) follow
VAR_LDS = 1           # LDS-resident scene, phase-aligned schedule, >= 7 waves/SIMD
VAR_LDS_ANY_OCC = 2   # ... without the occupancy target
VAR_GLOBAL = 3        # scene in HBM: quantised BVH4, LDS stack + global spill, suspended tails
VAR_MIS = (4, 5)      # MIS estimator: LDS scene, global scene
VAR_LDS6 = 6          # VAR_LDS built for >= 6 waves/SIMD (LDS copies that fit 6 but not 7 blocks per CU)
VAR_LDS_POOL = 7      # LDS-resident scene, block-pooled shadow queries (trace_kernel_pool)
VAR_LDS_POOL6 = 8     # VAR_LDS_POOL built for >= 6 waves/SIMD
VAR_REFERENCE = (VAR_LDS, VAR_LDS_ANY_OCC, VAR_GLOBAL, VAR_LDS6, VAR_LDS_POOL, VAR_LDS_POOL6)
VAR_POOL = (VAR_LDS_POOL, VAR_LDS_POOL6)
# ids 9-14 (round 5's fused / packed-leaf / split-arrival pooled schedules) were removed in round 6
VAR_LAST = 8
PRT_HITS_ANY = 0x1
PRT_HITS_QUANTIZED = 0x2

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64


class PrtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libprt error {code}: {msg}")
        self.code = code


_lib = None

EXPORTS = {
    "prt_abi_version": (_i, []),
    "prt_last_error": (ctypes.c_char_p, []),
    "prt_device_count": (_i, [_vp]),
    "prt_bvh_build": (_i, [_vp, _i64, _i32, _vp]),
    "prt_bvh_info": (_i, [_vp, _vp]),
    "prt_bvh_export": (_i, [_vp, _vp, _vp, _vp]),
    "prt_bvh_destroy": (None, [_vp]),
    "prt_scene_create": (_i, [_i, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _i32, _vp, _vp, _i32, _vp, _vp]),
    "prt_scene_info": (_i, [_vp, _vp]),
    "prt_scene_kernel": (_i, [_vp, _vp]),
    "prt_launch_kernel": (_i, [_vp, _i64, _u32, _vp]),
    "prt_closest_hits": (_i, [_vp, _vp, ctypes.c_int64, _u32, _vp, _vp]),
    "prt_hit_all": (_i, [_vp, _vp, _i64, _u64, _u32, _vp]),
    "prt_trace_rays": (_i, [_vp, _vp, _i64, _i, _u64, _u32, _vp]),
    "prt_scene_destroy": (None, [_vp]),
    "prt_render_tiles": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _u64, _u32, _vp, _vp]),
    "prt_render": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _u64, _u32, _vp, _vp]),
    "prt_render_multi": (_i, [_vp, _i, _vp, _i, _i, _i, _i, _i, _u64, _u32, _vp]),
    "prt_comm_release": (None, []),
    "prt_scatter_tiles": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "prt_scatter_frames": (_i, [_vp, _vp, _vp, _i, _i, _i64, _i, _i, _i, _i, _i, _i64, _vp, _vp]),
    "prt_camera_rays": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _u64, _vp]),
    "prt_render_tiles_device": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _u64, _u32, _vp, _vp]),
    "prt_render_frames_device": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _u64, _i, _i, _u32, _vp, _i64, _vp]),
    "prt_render_tiles_accumulate": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _u64, _u32, _vp]),
    "prt_kernel_timing": (_i, [_vp, _vp, _vp]),
    "prt_selftest_rcp": (_i, [_i, _vp]),
    "prt_selftest_guards": (_i, [_i, _vp]),
    "prt_check_faults": (_i, [_vp]),
    "prt_last_stats": (_i, [_vp, _vp]),
    "prt_diag_stats": (_i, [_vp, _vp]),
    "prt_diag_words": (_i, [_vp, _vp, _i]),
}


def lib():
    """Load libprt.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise PrtError(-100, f"{LIB} not found — run `python -m pyrenderer_amd.build` (hipcc, gfx950)")
        # torch-ROCm ships its own libamdhip64.so.7 with the same SONAME as /opt/rocm's:
        # whichever loads first serves the whole process.  Load torch first (when it is
        # installed) so that libprt and torch share ONE HIP runtime — torch streams and
        # device pointers handed to libprt are then valid, and torch can still see the GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.prt_abi_version() != ABI_VERSION:
            raise PrtError(-101, "ABI version mismatch")
        _lib = L
    return _lib


def check(rc):
    if rc != PRT_OK:
        raise PrtError(rc, lib().prt_last_error().decode(errors="replace"))
    return rc


def ptr(a):
    return None if a is None else a.ctypes.data_as(_vp)


def device_count():
    n = ctypes.c_int(0)
    check(lib().prt_device_count(ctypes.byref(n)))
    return n.value


class Bvh:
    """Host BVH (prt_bvh_build): for tests / inspection; scenes build their own."""

    def __init__(self, tri_v, max_leaf=4):
        tv = np.ascontiguousarray(tri_v, np.float32).reshape(-1, 9)
        h = _vp()
        check(lib().prt_bvh_build(ptr(tv), tv.shape[0], max_leaf, ctypes.byref(h)))
        self.h = h
        info = np.zeros(6, np.int64)
        check(lib().prt_bvh_info(self.h, ptr(info)))
        self.n_nodes, self.depth, self.n_leaves, self.n_tri = (int(x) for x in info[:4])
        self.pad = float(np.array([info[4]], np.int32).view(np.float32)[0])
        self.sah_cost = info[5] / 1000.0

    def export(self):
        nodes = np.zeros((self.n_nodes, 16), np.float32)
        tris = np.zeros((self.n_tri, 12), np.float32)
        order = np.zeros(self.n_tri, np.int32)
        check(lib().prt_bvh_export(self.h, ptr(nodes), ptr(tris), ptr(order)))
        return nodes, tris, order

    def __del__(self):
        if getattr(self, "h", None):
            lib().prt_bvh_destroy(self.h)
            self.h = None
