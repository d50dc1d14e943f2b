"""Ray sets of config 4 (the 1,000,044-triangle instanced cube.obj scene) for the coherence model
(tools/coherence_c4.cpp).

Follows PathTracer.trace's path structure (/root/reference/core/tracing.py:116-155) for one sample of
every pixel in a window of the 512 x 512 frame: the camera ray (main_taichi.py:89-95, the host
gen_ray), then per bounce the closest hit (the oracle's BVH backend), a cosine-hemisphere scatter
about the shading normal and one NEE shadow ray to a uniform point of the light (tracing.py:92-108).
Statistical, not bit-exact: the draws come from numpy, not from the kernels' keyed streams — the
model only needs rays distributed like the kernel's.  Output: a flat float32 file of records
(o.xyz, d.xyz, t_max, kind) with kind = 8 * bounce + (0 extension | 1 shadow) and the record's
pixel index, in pixel order within each (bounce, kind) — the order the kernel's pixel-major chunks
hand rays to waves.

    python tools/c4_rays.py --x0 192 --y0 192 --w 128 --h 128 --out /tmp/c4_rays.f32
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--x0", type=int, default=192)
    ap.add_argument("--y0", type=int, default=192)
    ap.add_argument("--w", type=int, default=128)
    ap.add_argument("--h", type=int, default=128)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="/tmp/c4_rays.f32")
    ap.add_argument("--scene", default="cubes", choices=("cubes", "cornell"),
                    help="config 4's instanced cubes (default) or the Cornell box of configs 1, 2 and 5")
    a = ap.parse_args()
    from oracle import oracle as O
    from pyrenderer_amd import scenes
    from pyrenderer_amd._native import Bvh
    from pyrenderer_amd.flatten import flatten_scene
    if a.scene == "cornell":
        from pyrenderer_amd.io_utils.read_tungsten import read_file
        scene, camera = read_file(scenes.CORNELL)
    else:
        scene, camera = scenes.instanced_cubes()
    flat = flatten_scene(scene)
    flat.tri_v.astype(np.float32).tofile(os.path.splitext(a.out)[0] + "_soup.f32")
    osc = O.OracleScene.from_flat(flat)
    nodes, _, order = Bvh(flat.tri_v).export()
    osc.set_bvh(nodes, order)
    pc = camera.convert_to_taichi_camera()
    W = H = 512
    rng = np.random.default_rng(a.seed)
    # pixels in the kernels' slot order for 64 x 64 tiles: tile-major, row-major inside a tile
    xs, ys = [], []
    for ty in range(a.y0 // 64, (a.y0 + a.h) // 64):
        for tx in range(a.x0 // 64, (a.x0 + a.w) // 64):
            yy, xx = np.mgrid[0:64, 0:64]
            xs.append((tx * 64 + xx).reshape(-1))
            ys.append((ty * 64 + yy).reshape(-1))
    px, py = np.concatenate(xs), np.concatenate(ys)
    pix = (py * W + px).astype(np.int64)
    u = ((px + rng.random(px.size)) / (W - 1)).astype(np.float32)
    v = ((py + rng.random(py.size)) / (H - 1)).astype(np.float32)
    o, d = pc.gen_ray(u, v)
    o, d = o.astype(np.float64), d.astype(np.float64)
    alive = np.arange(px.size)
    tv = flat.tri_v.reshape(-1, 3, 3).astype(np.float64)
    lt = flat.light_tri
    emit = flat.mat[flat.tri_mat, 3] != 0
    recs = []

    def put(oo, dd, tmax, kind, pp):
        r = np.zeros((oo.shape[0], 8), np.float32)
        r[:, 0:3], r[:, 3:6], r[:, 6] = oo, dd, tmax
        r[:, 7] = np.float32(kind)
        recs.append((r, pp))

    for b in range(a.depth):
        if alive.size == 0:
            break
        oo, dd = o[alive], d[alive]
        put(oo, dd, 1e10, 8 * b, pix[alive])
        hit, t, tri, nrm = osc.closest(oo.astype(np.float32), dd.astype(np.float32), 1e-5, 1e10, O.BACKEND_BVH)
        keep = (hit != 0) & ~emit[np.maximum(tri, 0)]
        alive, oo, dd, t, tri, nrm = alive[keep], oo[keep], dd[keep], t[keep], tri[keep], nrm[keep].astype(np.float64)
        p = oo + dd * t[:, None].astype(np.float64)
        # NEE: a uniform point of a random light triangle, the shadow ray bounded by the light
        k = lt[rng.integers(0, lt.size, p.shape[0])]
        su, sv = np.sqrt(rng.random(p.shape[0])), rng.random(p.shape[0])
        p2 = (tv[k, 0] * (su * (1 - sv))[:, None] + tv[k, 1] * (su * sv)[:, None] + tv[k, 2] * (1 - su)[:, None])
        w = p2 - p
        dist = np.linalg.norm(w, axis=1)
        w /= dist[:, None]
        vis = (w * nrm).sum(1) > 0
        put(p[vis], w[vis], dist[vis], 8 * b + 1, pix[alive[vis]])
        # cosine-hemisphere scatter about the shading normal
        r1, r2 = rng.random(p.shape[0]), rng.random(p.shape[0])
        phi, sr = 2 * np.pi * r1, np.sqrt(r2)
        lx, ly, lz = sr * np.cos(phi), sr * np.sin(phi), np.sqrt(1 - r2)
        up = np.where(np.abs(nrm[:, 1:2]) < 0.9, np.array([[0.0, 1.0, 0.0]]), np.array([[1.0, 0.0, 0.0]]))
        tx_ = np.cross(up, nrm)
        tx_ /= np.linalg.norm(tx_, axis=1, keepdims=True)
        ty_ = np.cross(nrm, tx_)
        nd = tx_ * lx[:, None] + ty_ * ly[:, None] + nrm * lz[:, None]
        o[alive], d[alive] = p, nd / np.linalg.norm(nd, axis=1, keepdims=True)
    r = np.concatenate([x for x, _ in recs])
    pp = np.concatenate([y for _, y in recs]).astype(np.float32)
    out = np.concatenate([r, pp[:, None]], axis=1)   # 9 floats: o, d, t_max, kind, pixel
    out.astype(np.float32).tofile(a.out)
    kinds, counts = np.unique(r[:, 7].astype(int), return_counts=True)
    print({"rays": int(r.shape[0]), "pixels": int(px.size), "by_kind": dict(zip(kinds.tolist(), counts.tolist()))})


if __name__ == "__main__":
    main()
