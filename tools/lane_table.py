"""Per-phase SIMD lane utilisation of the block-pooled trace kernel (diagnostic, round 5).

The STATS build of trace_kernel_pool books, for each phase, the wave-level trips of its loop body
(counted once per wave by the first active lane) and the lanes active in them (diag words 160..175):

    E inner / E leaf   extension traversal: inner-node visits, triangle tests
    S inner / S leaf   pooled shadow traversal: inner-node visits, triangle tests
    shade              the shading block (lanes that traversed in E)
    lambert            the Lambertian block inside it (cosine draw, frame, NEE sample, pre-test)
    iteration          one loop iteration (lanes holding a path after the refill)
    resolve            lanes resolving a pooled shadow answer

lanes = lane trips / (64 x wave trips).  With --clocks <lib built with -D PRT_POOL_CLOCKS>, the
wave-cycle split of the same render (tools/pool_clocks.py's phases) is added.  One process, one
full frame of the chosen config (default: config 2, variant 7 = trace_kernel_pool).

    python tools/lane_table.py [--config 2] [--clocks abtmp/libprt_clk.so] > profiles/r05/lanes/c2.json
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ("E_inner", "E_leaf", "S_inner", "S_leaf", "shade", "lambert", "iteration", "resolve")


def render_words(L, N, flat, cam, cfg, variant, flags, n_words=192):
    from pyrenderer_amd.device_scene import interleaved_tiles
    h = ctypes.c_void_p()
    sph = flat.sph if flat.sph.shape[0] else None
    N.check(L.prt_scene_create(0, N.ptr(flat.tri_v), N.ptr(flat.tri_n), N.ptr(flat.tri_mat), flat.n_tri, N.ptr(sph),
                               N.ptr(flat.sph_mat if sph is not None else None), flat.sph.shape[0], N.ptr(flat.mat),
                               flat.mat.shape[0], N.ptr(flat.light_tri), N.ptr(flat.light_off), flat.n_light,
                               N.ptr(flat.direct_rgb), ctypes.byref(h)))
    W = H = cfg["res"]
    ids = np.ascontiguousarray(interleaved_tiles(W, H, 64), np.int32)
    out = np.zeros((len(ids) * 64 * 64, 3), np.float32)
    st = np.zeros(4, np.uint64)
    for f in flags:
        N.check(L.prt_render_tiles(h, N.ptr(cam), W, H, 64, 64, N.ptr(ids), len(ids), cfg["spp"], cfg["depth"], 0,
                                   f | (variant << 8), N.ptr(out), N.ptr(st)))
    w = np.zeros(n_words, np.uint64)
    N.check(L.prt_diag_words(h, N.ptr(w), n_words))
    L.prt_scene_destroy(h)
    return w, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--variant", type=int, default=7)
    ap.add_argument("--clocks", help="libprt copy built with -D PRT_POOL_CLOCKS (adds the wave-cycle split)")
    a = ap.parse_args()
    import bench
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.flatten import flatten_scene
    L = N.lib()
    cfg = bench.CONFIGS[a.config]
    scene, camera = bench.load_scene(cfg["scene"])
    flat = flatten_scene(scene)
    cam = np.ascontiguousarray(camera.convert_to_taichi_camera().packed(), np.float32)
    w, img = render_words(L, N, flat, cam, cfg, a.variant, (N.PRT_FLAG_STATS,))
    samples = cfg["res"] * cfg["res"] * cfg["spp"]
    lt = w[160:176].astype(np.float64)
    table = {}
    for i, name in enumerate(PHASES):
        wt, lt_ = lt[2 * i], lt[2 * i + 1]
        table[name] = {"wave_trips_per_sample": round(wt / samples, 4),
                       "lanes": round(lt_ / (64.0 * wt), 4) if wt else None}
    res = {"config": a.config, "variant": a.variant, "samples": samples,
           "nodes_per_sample": round(float(w[0]) / samples, 3), "tris_per_sample": round(float(w[1]) / samples, 3),
           "ext_queries_per_sample": round(float(w[2]) / samples, 4),
           "shadow_rays_per_sample": round(float(w[3]) / samples, 4),
           "answered_by_light_test_per_sample": round(float(w[20]) / samples, 4),
           "lane_table": table}
    if a.clocks:
        from tools.ab_builds import load
        Lc = load(a.clocks)
        wc, _ = render_words(Lc, N, flat, cam, cfg, a.variant, (N.PRT_FLAG_STATS, 0), n_words=32)
        ck = wc[24:30].astype(np.float64)
        names = ("E_shade_enqueue", "barrier", "S", "unused", "E_refill", "E_traversal")
        tot = ck.sum()
        res["wave_cycle_split"] = {k: round(float(v / tot), 4) for k, v in zip(names, ck) if k != "unused"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
