"""Config 4's BVH, pinned independently of the oracle.

The config-4 frame test's oracle walks the BVH2 the library built (tests/test_gpu_configs.py), so a
builder bug that left part of a triangle outside its references' boxes would make GPU and oracle
agree.  Here the default large-scene tree (spatial splits + treelet restructuring + 64 SAH bins:
PRT_SBVH / PRT_TREELET / PRT_SAH_BINS unset, the tree prt_scene_create builds with max_leaf 4) of the
1,000,044-triangle instanced cube.obj scene is checked against the geometry alone: every triangle is
referenced, every reference slot lies in exactly one leaf, each reference's record is its triangle,
and EVERY triangle's three vertices and nine interior barycentric points lie inside the box of at
least one of its references — the property the conservative hit_aabb of
/root/reference/accelerators/bvh_taichi.py:168-190 needs for traversal to find every hit.  Inner
boxes nest: each node's box (in its parent) contains both of its child boxes.  Numpy, vectorised.
"""
import numpy as np
import pytest

from pyrenderer_amd import scenes
from pyrenderer_amd._native import Bvh
from pyrenderer_amd.flatten import flatten_scene

KNOBS = ("PRT_SBVH", "PRT_TREELET", "PRT_SAH_BINS", "PRT_ESC_BETA", "PRT_SBVH_ALPHA", "PRT_SBVH_BUDGET",
         "PRT_SAH_CT", "PRT_LEAF_MIN", "PRT_MAX_LEAF")


@pytest.fixture(scope="module")
def c4_tree():
    import os
    saved = {k: os.environ.pop(k) for k in KNOBS if k in os.environ}
    try:
        scene, _ = scenes.instanced_cubes()
        tv = flatten_scene(scene).tri_v.reshape(-1, 9)
        b = Bvh(tv)
        nodes, tris, order = b.export()
    finally:
        os.environ.update(saved)
    return tv, b, nodes, tris, order


def _child(nodes, side):
    bx = nodes[:, 6 * side:6 * side + 6].astype(np.float64)
    return bx[:, [0, 2, 4]], bx[:, [1, 3, 5]], nodes[:, 12 + side].view(np.int32)


def test_config4_tree_shape(c4_tree):
    tv, b, nodes, tris, order = c4_tree
    n = tv.shape[0]
    assert n == 1_000_044
    assert b.n_tri == order.shape[0] and b.n_nodes == nodes.shape[0] and 1 <= b.depth <= 64   # n_tri: references
    # spatial splits duplicate some references (budget 1.3 x): every triangle at least once
    assert np.bincount(order, minlength=n).min() >= 1 and n < order.shape[0] <= 1.3 * n + 1
    # each reference record is its whole triangle: v0 and the f32 edges, id bits in v0.w
    np.testing.assert_array_equal(tris[:, 0:3], tv[order, 0:3])
    np.testing.assert_array_equal(tris[:, 4:7], tv[order, 3:6] - tv[order, 0:3])
    np.testing.assert_array_equal(tris[:, 8:11], tv[order, 6:9] - tv[order, 0:3])
    np.testing.assert_array_equal(tris[:, 3].view(np.int32), order)
    # every inner node is reached exactly once, and every node's child boxes lie inside its own box
    refs = nodes[:, 12:14].view(np.int32)
    inner = refs[refs >= 0]
    assert np.array_equal(np.sort(inner), np.arange(1, nodes.shape[0]))
    for side in (0, 1):
        lo, hi, r = _child(nodes, side)
        k = np.nonzero(r >= 0)[0]
        for s2 in (0, 1):
            clo, chi, _ = _child(nodes[r[k]], s2)
            empty = (clo > chi).any(axis=1)          # an empty child box (inverted) holds nothing
            assert np.all(((clo >= lo[k]) & (chi <= hi[k])).all(axis=1) | empty)


def test_config4_every_triangle_covered_by_its_references(c4_tree):
    tv, b, nodes, tris, order = c4_tree
    n, n_ref = tv.shape[0], order.shape[0]
    # leaf slots -> their boxes (the box stored for the leaf in its parent)
    slot_lo = np.full((n_ref, 3), np.inf)
    slot_hi = np.full((n_ref, 3), -np.inf)
    seen = np.zeros(n_ref, np.int32)
    for side in (0, 1):
        lo, hi, r = _child(nodes, side)
        k = np.nonzero(r < 0)[0]
        v = -r[k].astype(np.int64) - 1
        first, cnt = v >> 3, (v & 7) + 1
        slots = np.repeat(first, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        leaf = np.repeat(k, cnt)
        np.add.at(seen, slots, 1)
        slot_lo[slots], slot_hi[slots] = lo[leaf], hi[leaf]
    assert (seen == 1).all(), "every reference slot belongs to exactly one leaf"
    # sample points: the vertices and nine interior barycentric points, in float64
    w = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [1 / 3, 1 / 3, 1 / 3], [0.5, 0.5, 0], [0, 0.5, 0.5],
                  [0.5, 0, 0.5], [0.8, 0.1, 0.1], [0.1, 0.8, 0.1], [0.1, 0.1, 0.8], [0.6, 0.3, 0.1],
                  [0.05, 0.25, 0.7]])
    covered = np.zeros((n, w.shape[0]), bool)
    for a in range(0, n_ref, 1 << 18):
        s = np.arange(a, min(n_ref, a + (1 << 18)))
        t = order[s]
        v = tv[t].reshape(-1, 3, 3).astype(np.float64)
        p = np.einsum("mk,nkc->nmc", w, v)                          # (slots, points, xyz)
        inside = ((p >= slot_lo[s, None, :]) & (p <= slot_hi[s, None, :])).all(axis=2)
        np.logical_or.at(covered, t, inside)
    bad = np.argwhere(~covered)
    assert bad.size == 0, (bad.shape[0], bad[:5])
