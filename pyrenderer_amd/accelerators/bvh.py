"""BVH over triangles (replaces accelerators/bvh_taichi.py's primitive BVH).

Built natively by libprt (pyrenderer_amd/csrc/prt_bvh.cpp: binned SAH, BVH2,
64-B nodes with both child boxes); `BVH(tri_v).export()` exposes the arrays.
"""
from .._native import Bvh as BVH  # noqa: F401
