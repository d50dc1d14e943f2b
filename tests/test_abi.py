"""libprt's C-ABI: the library loads without a GPU, exports every symbol that
include/prt.h declares, and its host-side BVH builder is sound."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "prt.h")).read()
    return sorted(set(re.findall(r"\b(prt_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from pyrenderer_amd import _native as N
    L = N.lib()
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(N.EXPORTS), set(names) ^ set(N.EXPORTS)
    assert L.prt_abi_version() == N.ABI_VERSION == 4


def test_device_count_without_gpu_is_ok():
    from pyrenderer_amd import _native as N
    assert N.device_count() >= 0


def test_errors_are_reported():
    import ctypes
    from pyrenderer_amd import _native as N
    h = ctypes.c_void_p()
    rc = N.lib().prt_bvh_build(None, 5, 4, ctypes.byref(h))
    assert rc == -1 and b"NULL" in N.lib().prt_last_error()
    with pytest.raises(N.PrtError):
        N.Bvh(np.zeros((2, 9), np.float32), max_leaf=0)


def test_scatter_frames_rejects_overlapping_groups():
    """with several groups, a group_pitch shorter than its n_frames frames at src_frame_pitch
    would let frame f of group g read group g + 1's block; the shape check rejects it before any device
    work (no scene or GPU needed to reach it)."""
    from pyrenderer_amd import _native as N
    L = N.lib()
    ids = np.zeros(2, np.int32)
    slot = 16 * 16 * 3
    # 2 groups of 1 tile, 2 frames at a pitch of one slot: a group needs 2 slots
    rc = L.prt_scatter_frames(None, None, N.ptr(ids), 2, 1, slot, 16, 16, 32, 32, 2, slot, None, None)
    assert rc == -1 and b"n_frames frames" in L.prt_last_error()   # PRT_ERR_ARG


def _traverse_py(nodes, tris, order, ro, rd, tmin, tmax):
    """Brute-force over the leaves reachable through conservative boxes (python)."""
    import struct

    def ref(f):
        return struct.unpack("<i", struct.pack("<f", f))[0]

    found = []
    stack = [0]
    inv = 1.0 / np.where(rd == 0, 1e-30, rd)
    while stack:
        cur = stack.pop()
        if cur >= 0:
            n = nodes[cur]
            for side, c in ((0, ref(n[12])), (1, ref(n[13]))):
                b = n[6 * side:6 * side + 6]
                lo = np.array([b[0], b[2], b[4]])
                hi = np.array([b[1], b[3], b[5]])
                t0 = (lo - ro) * inv
                t1 = (hi - ro) * inv
                tn = np.max(np.minimum(t0, t1))
                tf = np.min(np.maximum(t0, t1))
                if max(tn, tmin) <= min(tf, tmax) * (1 + 1e-6):
                    stack.append(c)
        else:
            v = -cur - 1
            first, cnt = v >> 3, (v & 7) + 1
            found.extend(order[first:first + cnt].tolist())
    return set(found)


@pytest.mark.parametrize("sbvh,treelet", [("0", "0"), ("1", "0"), ("1", "3"), ("0", "3")])
def test_bvh_build_covers_every_triangle_with_conservative_boxes(sbvh, treelet, monkeypatch):
    """Object splits only (PRT_SBVH=0): the leaves partition the triangles and every leaf triangle lies
    inside its child box.  With spatial splits (the default, prt_bvh.cpp) a triangle may have several
    references, each bounding its part of the triangle: every triangle is referenced, and every point of
    it lies inside the box of one of its references.  Treelet restructuring (PRT_TREELET passes) only
    rearranges inner nodes: the same guarantees hold, and the SAH cost does not rise."""
    from pyrenderer_amd import _native as N
    monkeypatch.setenv("PRT_SBVH", sbvh)
    monkeypatch.setenv("PRT_TREELET", treelet)
    rng = np.random.default_rng(3)
    n = 3000
    c = rng.uniform(-5, 5, (n, 1, 3))
    tv = (c + rng.normal(0, 0.2, (n, 3, 3))).astype(np.float32).reshape(n, 9)
    b = N.Bvh(tv, max_leaf=4)
    if treelet != "0":
        monkeypatch.setenv("PRT_TREELET", "0")
        assert b.sah_cost <= N.Bvh(tv, max_leaf=4).sah_cost + 1e-9
    nodes, tris, order = b.export()
    if sbvh == "0":
        assert sorted(order.tolist()) == list(range(n))
    else:
        assert set(order.tolist()) == set(range(n)) and n <= len(order) <= 1.3 * n + 1
    assert 1 <= b.depth <= 64
    # triangle records: v0 and f32 edges, original id in v0.w bits
    np.testing.assert_array_equal(tris[:, 0:3], tv[order, 0:3])
    np.testing.assert_array_equal(tris[:, 4:7], tv[order, 3:6] - tv[order, 0:3])
    np.testing.assert_array_equal(tris[:, 3].view(np.int32), order)
    # leaf boxes: whole triangles (object splits) / a cover of each triangle by its references' boxes
    import struct
    boxes = {}
    for nd in nodes:
        for side in (0, 1):
            r = struct.unpack("<i", struct.pack("<f", nd[12 + side]))[0]
            if r < 0:
                v = -r - 1
                first, cnt = v >> 3, (v & 7) + 1
                bx = nd[6 * side:6 * side + 6]
                lo, hi = np.array([bx[0], bx[2], bx[4]]), np.array([bx[1], bx[3], bx[5]])
                for t in order[first:first + cnt]:
                    boxes.setdefault(int(t), []).append((lo, hi))
                if sbvh == "0":
                    pts = tv[order[first:first + cnt]].reshape(-1, 3)
                    assert np.all(pts >= lo) and np.all(pts <= hi)
    w = rng.dirichlet((1, 1, 1), 12)
    for t in range(0, n, 7):
        v = tv[t].reshape(3, 3).astype(np.float64)
        for p in np.concatenate([v, w @ v]):
            assert any(np.all(p >= lo) and np.all(p <= hi) for lo, hi in boxes[t]), (t, p)
    # rays: the brute-force closest triangle is among the reachable leaves
    from oracle import oracle as O
    osc = O.OracleScene(tv, np.tile([0, 1, 0], (n, 1)), np.zeros(n), np.arange(n), tv[:, :3], tv[:, :3],
                        np.array([[1, 1, 1, 0, 0, 0, 1, 0]]), [0], [0, 1], [1, 1, 1])
    ro = rng.uniform(-6, 6, (300, 3)).astype(np.float32)
    rd = rng.normal(size=(300, 3))
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    hit, t, tri, _ = osc.closest(ro, rd, 1e-5, 1e5, O.BACKEND_BRUTE)
    assert hit.sum() > 50
    for i in np.nonzero(hit)[0][:80]:
        assert tri[i] in _traverse_py(nodes, tris, order, ro[i].astype(np.float64), rd[i].astype(np.float64), 1e-5, 1e5)


@pytest.mark.parametrize("treelet", ["0", "3"])
def test_bvh_depth_is_the_exported_trees_depth(treelet, monkeypatch):
    """The depth prt_bvh_info reports (it sizes the traversal stacks) is the exported BVH2's, also after
    treelet restructuring has moved inner nodes (prt_bvh.cpp tree_depth); every inner node is reached
    once from the root."""
    import struct
    from pyrenderer_amd import _native as N
    monkeypatch.setenv("PRT_TREELET", treelet)
    rng = np.random.default_rng(11)
    n = 5000
    c = rng.uniform(-5, 5, (n, 1, 3)) * rng.uniform(0.2, 1.0, (n, 1, 3)) ** 2
    tv = (c + rng.normal(0, 0.05, (n, 3, 3))).astype(np.float32).reshape(n, 9)
    b = N.Bvh(tv, max_leaf=4)
    nodes, _, _ = b.export()
    seen = np.zeros(len(nodes), np.int32)
    deepest, stack = 0, [(0, 0)]
    while stack:
        i, d = stack.pop()
        seen[i] += 1
        for side in (0, 1):
            r = struct.unpack("<i", struct.pack("<f", nodes[i][12 + side]))[0]
            if r >= 0:
                stack.append((r, d + 1))
            else:
                deepest = max(deepest, d + 1)
    assert (seen == 1).all()
    assert b.depth == deepest


def test_bvh_degenerate_inputs():
    from pyrenderer_amd import _native as N
    b = N.Bvh(np.zeros((0, 9), np.float32))
    assert b.n_nodes == 1
    one = N.Bvh(np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0]], np.float32))
    nodes, tris, order = one.export()
    assert one.n_nodes == 1 and order.tolist() == [0]
    same = N.Bvh(np.tile(np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0]], np.float32), (50, 1)))
    assert sorted(same.export()[2].tolist()) == list(range(50))
    with pytest.raises(N.PrtError):
        N.Bvh(np.full((1, 9), np.nan, np.float32))


def test_window_and_multi_argument_errors_without_gpu():
    """prt_render / prt_render_multi reject bad handles and shapes before touching a device."""
    import ctypes
    from pyrenderer_amd import _native as N
    L = N.lib()
    cam = np.zeros(24, np.float32)
    out = np.zeros((4, 4, 3), np.float32)
    assert L.prt_render(None, N.ptr(cam), 4, 4, 0, 0, 4, 4, 1, 1, 0, 0, N.ptr(out), None) == -1
    assert b"NULL" in L.prt_last_error()
    assert L.prt_render_multi(None, 1, N.ptr(cam), 4, 4, 8, 1, 1, 0, 0, N.ptr(out)) == -1
    hs = (ctypes.c_void_p * 2)(None, None)
    assert L.prt_render_multi(hs, 0, N.ptr(cam), 4, 4, 8, 1, 1, 0, 0, N.ptr(out)) == -1
    assert L.prt_render_multi(hs, 2, N.ptr(cam), 4, 4, 8, 1, 1, 0, 0, N.ptr(out)) == -1
    assert b"NULL" in L.prt_last_error()
    L.prt_comm_release()   # no communicator yet: a no-op



def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: without libprt.so every product entry point raises."""
    from pyrenderer_amd import _native as N
    monkeypatch.setattr(N, "LIB", str(tmp_path / "libprt.so"))
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(N.PrtError, match="not found"):
        N.lib()
    with pytest.raises(N.PrtError):
        N.device_count()
