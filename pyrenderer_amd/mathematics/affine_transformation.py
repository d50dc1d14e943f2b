"""Tungsten transform → 4x4 matrix (reference: mathematics/affine_transformation.py:7-55).

res = T @ Rx @ Ry @ Rz @ S (column vectors).  dtype flow mirrors the reference
exactly: T and S are float32 (so JSON positions/scales are rounded to f32
first), per-axis rotations are float64 (scipy Rotation.from_euler, one axis at a
time, degrees), products promote to float64 once a rotation is involved.
"""
import numpy as np

try:
    from scipy.spatial.transform import Rotation as _Rotation
except Exception:  # pragma: no cover - scipy is part of the image
    _Rotation = None


def _axis_rotation(axis, degree):
    if _Rotation is not None:
        return _Rotation.from_euler(axis, degree, degrees=True).as_matrix()
    # scipy's quaternion route: q = (sin(h) e_axis, cos(h)), h = theta/2
    h = np.radians(degree) / 2.0
    q = np.zeros(4)
    q["xyz".index(axis)] = np.sin(h)
    q[3] = np.cos(h)
    x, y, z, w = q / np.linalg.norm(q)
    return np.array([[x * x - y * y - z * z + w * w, 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), -x * x + y * y - z * z + w * w, 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), -x * x - y * y + z * z + w * w]])


def to_homogeneous_matrix(mat):
    res = np.hstack([mat, np.zeros((3, 1))])
    res = np.vstack([res, np.zeros((4,))])
    res[3][3] = 1.0
    return res


def make_rotation_matrix(degrees, homo=True):
    rot_mat = np.identity(3, np.float32)
    for d_id, degree in enumerate(degrees):
        if degree != 0:
            rot_mat = rot_mat @ _axis_rotation("xyz"[d_id], degree)
    return to_homogeneous_matrix(rot_mat) if homo else rot_mat


def make_translation_matrix(moves):
    res = np.identity(4, np.float32)
    res[:3, 3] = moves
    return res


def make_scale_matrix(scales):
    res = np.identity(4, np.float32)
    res[0, 0], res[1, 1], res[2, 2] = scales[0], scales[1], scales[2]
    return res


def make_transformation_matrix(transforms):
    """transforms: Tungsten `transform` dict with optional position/rotation/scale."""
    res = np.identity(4, np.float32)
    if "position" in transforms:
        res = res @ make_translation_matrix(transforms["position"])
    if "rotation" in transforms:
        res = res @ make_rotation_matrix(transforms["rotation"])
    if "scale" in transforms:
        res = res @ make_scale_matrix(transforms["scale"])
    return res
