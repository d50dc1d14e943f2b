"""Where the block-pooled kernel's waves spend their time (diagnostic): a library copy built with
-DPRT_POOL_CLOCKS accumulates wave-level s_memtime cycles per phase — E (refill / extension query /
shading + enqueue), waiting at barrier 1, S (pooled shadow queries, or the refill of waves without an S
chunk), waiting at barrier 2 — into diag words 24..29.  One process, config 2, variant 7.

    python -m pyrenderer_amd.build --out abtmp/libprt_clk.so -D PRT_POOL_CLOCKS
    python tools/pool_clocks.py --lib abtmp/libprt_clk.so
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--variant", type=int, default=7)
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    import bench
    from pyrenderer_amd import _native as N
    from tools.ab_builds import load
    N.lib()
    L = load(a.lib)
    from pyrenderer_amd.device_scene import interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    cfg = bench.CONFIGS[a.config]
    scene, camera = bench.load_scene(cfg["scene"])
    flat = flatten_scene(scene)
    cam = np.ascontiguousarray(camera.convert_to_taichi_camera().packed(), np.float32)
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
    for flags in (N.PRT_FLAG_STATS, 0):   # the STATS render zeroes the diag words, the clock build adds to 24..27
        N.check(L.prt_render_tiles(h, N.ptr(cam), W, H, 64, 64, N.ptr(ids), len(ids), cfg["spp"], cfg["depth"], 0,
                                   flags | (a.variant << 8), N.ptr(out), N.ptr(st)))
    w = np.zeros(30, np.uint64)
    N.check(L.prt_diag_words(h, N.ptr(w), 30))
    ck = w[24:30].astype(np.float64)
    tot = ck.sum()
    names = ("E_shade_enqueue", "barrier1", "S", "barrier2", "E_refill", "E_traversal")
    print(json.dumps({"variant": a.variant, "config": a.config, "wave_cycles": float(tot),
                      "frac": {k: round(float(v / tot), 4) for k, v in zip(names, ck)}}))
    L.prt_scene_destroy(h)


if __name__ == "__main__":
    main()
