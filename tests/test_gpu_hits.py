"""Hit-level GPU parity: `prt_closest_hits` (the kernels' BVH4 traversal, float and
quantised nodes, + spheres) against the oracle's brute-force `World.hit_all`
(mathematics/intersection_taichi.py:238-291) on the same rays, bit for bit.

Includes rays with direction components of exactly 0 (1/d = inf): the case where a
min/max slab formulation turns a NaN plane distance into a wrong cull.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

T_MIN, T_MAX = np.float32(1e-5), np.float32(99999.9)


def _rays(n, seed, lo=(-1.0, 0.0, -1.0), hi=(1.0, 2.0, 1.0)):
    rng = np.random.default_rng(seed)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    return o, d


def _axis_rays(n, seed, lo=(-1.0, 0.0, -1.0), hi=(1.0, 2.0, 1.0)):
    """Directions with exact zero components (axis-parallel and diagonal-in-plane),
    and -0.0 as well as +0.0."""
    rng = np.random.default_rng(seed)
    dirs = []
    s = np.float32(np.sqrt(np.float32(0.5)))
    for a in range(3):
        for sign in (1.0, -1.0):
            v = [0.0, 0.0, 0.0]
            v[a] = sign
            dirs.append(v)
            w = [-0.0, -0.0, -0.0]
            w[a] = sign
            dirs.append(w)
    for a, b in ((0, 1), (0, 2), (1, 2)):
        for sa in (1.0, -1.0):
            for sb in (1.0, -1.0):
                v = [0.0, 0.0, 0.0]
                v[a], v[b] = sa * s, sb * s
                dirs.append(v)
    dirs = np.array(dirs, np.float32)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    # some origins exactly on box-plane coordinates of the scene (walls at +-1, 0, 2)
    o[: n // 4, 0] = rng.choice(np.array([-1.0, 1.0, 0.0, 0.5], np.float32), n // 4)
    oo = np.repeat(o, len(dirs), axis=0)
    dd = np.tile(dirs, (n, 1))
    return oo, dd


def _check_closest(ds, osc, o, d, quantized=False):
    gid, gt = ds.closest_hits(o, d, T_MIN, T_MAX, quantized=quantized)
    hit, t, tri, _ = osc.closest(o, d, T_MIN, T_MAX)
    oid = np.where(hit != 0, tri, -1).astype(np.int64)
    bad = np.nonzero((gid != oid) | ((gid >= 0) & (gt != t)))[0]
    assert bad.size == 0, (bad.size, [(o[i], d[i], gid[i], oid[i], gt[i], t[i]) for i in bad[:5]])
    return (gid >= 0).mean()


def _check_any(ds, osc, o, d, tmax, quantized=False):
    gid, _ = ds.closest_hits(o, d, T_MIN, tmax, any_hit=True, quantized=quantized)
    hit, _, _, _ = osc.closest(o, d, T_MIN, tmax)
    assert np.array_equal(gid >= 0, hit != 0)


@pytest.mark.parametrize("quantized", [False, True])
def test_cornell_hits_match_oracle(gpu_scene, oracle_scene, quantized):
    o, d = _rays(20000, 1)
    frac = _check_closest(gpu_scene, oracle_scene, o, d, quantized)
    assert frac > 0.5
    o, d = _axis_rays(3000, 2)
    _check_closest(gpu_scene, oracle_scene, o, d, quantized)
    # shadow-style bounded queries
    o, d = _rays(20000, 3)
    tmax = np.random.default_rng(4).uniform(0.01, 3.0, o.shape[0]).astype(np.float32)
    _check_any(gpu_scene, oracle_scene, o, d, tmax, quantized)


@pytest.mark.parametrize("quantized", [False, True])
def test_soup_hits_match_oracle(cornell, quantized):
    from test_gpu_parity import _soup_scene
    from pyrenderer_amd.device_scene import DeviceScene
    flat = _soup_scene(cornell, 3000, 9)
    ds = DeviceScene(flat, 0)
    osc = O.OracleScene.from_flat(flat)
    o, d = _rays(20000, 5)
    _check_closest(ds, osc, o, d, quantized)
    o, d = _axis_rays(2000, 6)
    _check_closest(ds, osc, o, d, quantized)


def test_sphere_scene_hits_match_oracle():
    from test_gpu_parity import _specular_scene
    from pyrenderer_amd.device_scene import DeviceScene
    _, _, flat = _specular_scene(0.0)
    ds = DeviceScene(flat, 0)
    osc = O.OracleScene.from_flat(flat)
    o, d = _rays(20000, 7)
    _check_closest(ds, osc, o, d)
    o, d = _axis_rays(1000, 8)
    _check_closest(ds, osc, o, d)
