"""Pinhole camera (reference: core/camera.py:13-72, core/camera_taichi.py:10-74).

`view` is pyrr's look-at in its row-vector layout (restated here; pyrr is not
a dependency), `iview = inv(view)`.  `convert_to_taichi_camera()` returns the
packed f32 record the HIP kernel's gen_ray consumes (include/prt.h PRT_CAM_*):
  [0:16]  iview columns c1..c4 (= rows of iview.T, camera_taichi.py:100-107)
  [16:20] sensor_dim = (sensor_width, sensor_height, focus_dist, aperture)
          with sensor_height = tan(radians(fov)/2) * focus_dist (camera_taichi.py:108-111)
  [20:24] reserved (0)
"""
from math import radians, tan

import numpy as np


def create_look_at(eye, target, up):
    eye = np.asarray(eye, dtype=np.float64)
    target = np.asarray(target, dtype=np.float64)
    up = np.asarray(up, dtype=np.float64)

    def _n(v):
        return v / np.sqrt(np.sum(v * v))

    forward = _n(target - eye)
    side = _n(np.cross(forward, up))
    up = _n(np.cross(side, forward))
    return np.array(((side[0], up[0], -forward[0], 0.),
                     (side[1], up[1], -forward[1], 0.),
                     (side[2], up[2], -forward[2], 0.),
                     (-np.dot(side, eye), -np.dot(up, eye), np.dot(forward, eye), 1.0)))


class PackedCamera:
    """What CameraTaichi holds, as the 24-float C-ABI record."""

    def __init__(self, iview_mat, fov, aspect_ratio, aperture, focus_dist):
        cols = np.asarray(iview_mat, np.float64)  # = iview.T; row i is iview_c{i+1}
        sensor_height = tan(radians(fov) / 2) * focus_dist
        sensor_width = sensor_height * aspect_ratio
        self.iview_cols = cols.astype(np.float32)
        self.sensor_dim = np.array([sensor_width, sensor_height, focus_dist, aperture], np.float32)
        self.origin = cols[:, 3].astype(np.float32)

    def packed(self):
        out = np.zeros(24, np.float32)
        out[:16] = self.iview_cols.reshape(-1)
        out[16:20] = self.sensor_dim
        return out

    def gen_ray(self, u, v, lens=None):
        """CameraTaichi.gen_ray (core/camera_taichi.py:47-74), which the reference's render loop calls
        per sample (main_taichi.py:95): the ray through sensor coordinates (u, v) in [0, 1]^2, as
        (origin, direction) float32 arrays of shape (..., 3) for scalar or array u, v.

        f32 arithmetic in the reference's expression order — bit-identical to the kernel's gen_ray
        (camera_kernel) and the oracle's.  With an aperture the origin is jittered by two uniform
        draws per ray, as the reference's two rand() calls (the focus-distance scale kept):
        `lens` (..., 2) supplies them (the kernel draws them from the sample's stream after the pixel
        jitter); without it they come from numpy's default generator."""
        f = np.float32
        u = np.asarray(u, f)
        v = np.asarray(v, f)
        u, v = np.broadcast_arrays(u, v)
        sd = self.sensor_dim
        half = f(0.5)
        rd = [(u - half) * sd[0] / half, (v - half) * sd[1] / half, np.full(u.shape, -sd[2], f), np.ones(u.shape, f)]
        ro = [np.zeros(u.shape, f), np.zeros(u.shape, f), np.zeros(u.shape, f), np.ones(u.shape, f)]
        if sd[3] > 0:
            if lens is None:
                lens = np.random.default_rng().random(u.shape + (2,), dtype=f)
            lens = np.asarray(lens, f)
            ro[0] = sd[2] * lens[..., 0] - sd[2] / f(2.0)
            ro[1] = sd[2] * lens[..., 1] - sd[2] / f(2.0)
        c = self.iview_cols          # row i = iview_c{i+1}
        dw = [((rd[0] * c[i, 0] + rd[1] * c[i, 1]) + rd[2] * c[i, 2]) + rd[3] * c[i, 3] for i in range(4)]
        ow = [((ro[0] * c[i, 0] + ro[1] * c[i, 1]) + ro[2] * c[i, 2]) + ro[3] * c[i, 3] for i in range(4)]
        fr = [dw[i] - ow[i] for i in range(4)]
        ln = np.sqrt(((fr[0] * fr[0] + fr[1] * fr[1]) + fr[2] * fr[2]) + fr[3] * fr[3])
        origin = np.stack(ow[:3], axis=-1).astype(f)
        direction = np.stack([fr[0] / ln, fr[1] / ln, fr[2] / ln], axis=-1).astype(f)
        return origin, direction


class Camera:
    def __init__(self, position, looking_at, up, resolution, fov=90, aperture=0, focal_dist=1.0):
        self.position = np.array(position)
        self.looking_at = np.array(looking_at)
        self.up = np.array(up)
        self.view = create_look_at(self.position, self.looking_at, self.up)
        self.iview = np.linalg.inv(self.view)
        self.resolution = resolution
        self.aperture = aperture
        self.focal_dist = focal_dist
        self.fov = fov
        self.aspect_ratio = self.resolution[0] / self.resolution[1] * 1.0

    def convert_to_taichi_camera(self):
        aspect_ratio = float(self.resolution[0]) / self.resolution[1]
        return PackedCamera(self.iview.T, self.fov, aspect_ratio, self.aperture, self.focal_dist)

    def packed(self, resolution=None):
        """24-float camera record; `resolution` overrides the aspect ratio source."""
        res = resolution or self.resolution
        aspect_ratio = float(res[0]) / res[1]
        return PackedCamera(self.iview.T, self.fov, aspect_ratio, self.aperture, self.focal_dist).packed()

    def get_resolution(self):
        return self.resolution
