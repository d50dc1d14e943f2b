"""The host camera API: Camera.convert_to_taichi_camera() returns an object
with the reference's per-ray gen_ray(u, v) (core/camera_taichi.py:47-74, called per sample at
main_taichi.py:95), evaluated in numpy f32 in the reference's expression order.  Pinned bit for bit
to the vectors the reference's own gen_ray produced (tests/golden/kats.npz, tests/golden/gen/)."""
import copy

import numpy as np

from conftest import ROOT  # noqa: F401


def _kats():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "kats.npz"))


def test_gen_ray_equals_the_reference_vectors(cornell):
    k = _kats()
    pc = cornell[1].convert_to_taichi_camera()
    o, d = pc.gen_ray(k["cam_uv"][:, 0], k["cam_uv"][:, 1])
    assert o.dtype == np.float32 and d.dtype == np.float32 and d.shape == k["cam_d"].shape
    np.testing.assert_array_equal(o, k["cam_o"])
    np.testing.assert_array_equal(d, k["cam_d"])
    # scalars, the reference's call form
    for i in (0, 17, 999):
        o1, d1 = pc.gen_ray(float(k["cam_uv"][i, 0]), float(k["cam_uv"][i, 1]))
        assert o1.shape == (3,) and np.array_equal(o1, k["cam_o"][i]) and np.array_equal(d1, k["cam_d"][i])


def test_gen_ray_equals_the_oracle_for_general_cameras(cornell):
    """Thin-lens draws supplied per ray (`lens`) and a projective (non-affine) matrix: the same
    operations as the oracle's gen_ray (oracle/prt_oracle.c) for the affine case, and unit-length
    directions through the lens."""
    from oracle import oracle as O
    pc = cornell[1].convert_to_taichi_camera()
    rng = np.random.default_rng(5)
    uv = rng.random((300, 2), dtype=np.float32)
    proj = copy.deepcopy(pc)
    proj.iview_cols = proj.iview_cols.copy()
    proj.iview_cols[3, 0] = np.float32(1e-3)          # last row of iview != (0, 0, 0, 1)
    o, d = proj.gen_ray(uv[:, 0], uv[:, 1])
    for i in range(0, 300, 7):
        oo, dd = O.gen_ray(proj.packed(), *uv[i])
        assert np.array_equal(o[i], oo) and np.array_equal(d[i], dd), i
    lens = copy.deepcopy(pc)
    lens.sensor_dim = lens.sensor_dim.copy()
    lens.sensor_dim[3] = np.float32(1.0)
    xi = rng.random((300, 2), dtype=np.float32)
    o2, d2 = lens.gen_ray(uv[:, 0], uv[:, 1], lens=xi)
    o3, d3 = lens.gen_ray(uv[:, 0], uv[:, 1], lens=xi)
    assert np.array_equal(o2, o3) and np.array_equal(d2, d3)
    assert not np.array_equal(o2, np.broadcast_to(pc.origin[:3], o2.shape))   # jittered origins
    np.testing.assert_allclose(np.linalg.norm(d2.astype(np.float64), axis=1), 1.0, atol=1e-6)
