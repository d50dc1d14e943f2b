"""Flatten a host Scene into the arrays the C-ABI consumes (include/prt.h).

Mirrors what the reference bakes into Taichi fields at World.commit()
(mathematics/intersection_taichi.py:220-233, shapes.py:49-57): float32
world-space vertices, float32 face normals, the per-primitive BSDF, and the
light list (emitting primitives in insertion order, each with its faces for
Quad.sample_a_point's randInt face choice).
"""
import numpy as np

from .mathematics.constants import DIRECT_LIGHT_RGB


class FlatScene:
    def __init__(self, tri_v, tri_n, tri_mat, tri_prim, prim_lo, prim_hi, mat, light_tri, light_off,
                 direct_rgb=DIRECT_LIGHT_RGB, sph=None, sph_mat=None):
        self.tri_v = np.ascontiguousarray(tri_v, np.float32).reshape(-1, 9)
        self.tri_n = np.ascontiguousarray(tri_n, np.float32).reshape(-1, 3)
        self.tri_mat = np.ascontiguousarray(tri_mat, np.int32)
        self.tri_prim = np.ascontiguousarray(tri_prim, np.int32)
        self.prim_lo = np.ascontiguousarray(prim_lo, np.float32).reshape(-1, 3)
        self.prim_hi = np.ascontiguousarray(prim_hi, np.float32).reshape(-1, 3)
        self.mat = np.ascontiguousarray(mat, np.float32).reshape(-1, 8)
        self.light_tri = np.ascontiguousarray(light_tri, np.int32)
        self.light_off = np.ascontiguousarray(light_off, np.int32)
        self.direct_rgb = np.ascontiguousarray(direct_rgb, np.float32)
        self.sph = np.zeros((0, 4), np.float32) if sph is None else np.ascontiguousarray(sph, np.float32).reshape(-1, 4)
        self.sph_mat = np.zeros(0, np.int32) if sph_mat is None else np.ascontiguousarray(sph_mat, np.int32)

    @property
    def n_tri(self):
        return self.tri_v.shape[0]

    @property
    def n_light(self):
        return self.light_off.shape[0] - 1


def flatten_scene(scene):
    """Scene (core.scene.Scene) → FlatScene."""
    mats, mat_index = [], {}
    tri_v, tri_n, tri_mat, tri_prim, prim_lo, prim_hi = [], [], [], [], [], []
    sph, sph_mat = [], []
    light_tri, light_off = [], [0]
    base = 0
    for pid, prim in enumerate(scene.primitives):
        key = id(prim.bsdf)
        if key not in mat_index:
            mat_index[key] = len(mats)
            mats.append(prim.bsdf.pack())
        m = mat_index[key]
        lo, hi = prim.bounding_box
        prim_lo.append(np.asarray(lo, np.float32))
        prim_hi.append(np.asarray(hi, np.float32))
        if getattr(prim, "type_name", "") == "sphere":
            sph.append([*np.asarray(prim.center, np.float32), np.float32(prim.radius)])
            sph_mat.append(m)
            continue
        v32 = np.asarray(prim.vertices, np.float32)
        f = np.asarray(prim.faces, np.int64)
        nf = f.shape[0]
        tri_v.append(v32[f].reshape(nf, 9))
        tri_n.append(np.asarray(prim.normal_vectors, np.float32))
        tri_mat.append(np.full(nf, m, np.int32))
        tri_prim.append(np.full(nf, pid, np.int32))
        if prim.bsdf.emitting_light:
            light_tri.extend(range(base, base + nf))
            light_off.append(len(light_tri))
        base += nf
    if len(light_off) == 1:
        raise ValueError("There is no lights!!!")  # intersection_taichi.py:233
    return FlatScene(np.concatenate(tri_v) if tri_v else np.zeros((0, 9)), np.concatenate(tri_n) if tri_n else np.zeros((0, 3)),
                     np.concatenate(tri_mat) if tri_mat else np.zeros(0), np.concatenate(tri_prim) if tri_prim else np.zeros(0),
                     np.stack(prim_lo), np.stack(prim_hi), np.asarray(mats, np.float32), np.asarray(light_tri, np.int32),
                     np.asarray(light_off, np.int32), DIRECT_LIGHT_RGB,
                     np.asarray(sph, np.float32) if sph else None, np.asarray(sph_mat, np.int32) if sph_mat else None)
