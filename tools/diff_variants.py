"""Render a frame with two kernel variants; where they differ, re-render the
differing 8x8 tiles with the CPU oracle and report which variant matches it.

    python tools/diff_variants.py --a 15 --b 30 [--res 512 --spp 64 --depth 8]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", type=int, required=True)
    ap.add_argument("--b", type=int, required=True)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--max-tiles", type=int, default=16)
    a = ap.parse_args()
    from oracle import oracle as O
    from pyrenderer_amd.device_scene import DeviceScene, unpack_tiles
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    from pyrenderer_amd import scenes
    scene, cam = read_file(scenes.CORNELL)
    flat = flatten_scene(scene)
    ds = DeviceScene(flat, 0)
    c = cam.convert_to_taichi_camera().packed()
    W = H = a.res
    T = 8
    ids = np.arange((W // T) * (H // T), dtype=np.int32)
    ga, _ = ds.render_tiles(c, W, H, T, T, ids, a.spp, a.depth, 0, a.a << 8)
    gb, _ = ds.render_tiles(c, W, H, T, T, ids, a.spp, a.depth, 0, a.b << 8)
    ga = ga.reshape(len(ids), T * T, 3)
    gb = gb.reshape(len(ids), T * T, 3)
    bad = np.nonzero(np.any(ga != gb, axis=(1, 2)))[0]
    print("differing tiles:", len(bad), "pixels:", int(np.any(ga != gb, axis=2).sum()))
    osc = O.OracleScene.from_flat(flat)
    sel = bad[: a.max_tiles].astype(np.int32)
    if len(sel):
        o = osc.render_tiles(c, W, H, T, T, sel, a.spp, a.depth, seed=0).reshape(len(sel), T * T, 3)
        ma = np.all(o == ga[sel], axis=(1, 2))
        mb = np.all(o == gb[sel], axis=(1, 2))
        print("tiles matching oracle: a", int(ma.sum()), "b", int(mb.sum()), "of", len(sel))
        for i, t in enumerate(sel[:4]):
            px = np.nonzero(np.any(ga[t] != gb[t], axis=1))[0]
            for p in px[:3]:
                print(" tile", int(t), "px", int(p), "a", ga[t, p], "b", gb[t, p], "oracle", o[i, p])


if __name__ == "__main__":
    main()
