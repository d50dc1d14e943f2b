"""Render a small Cornell frame with a given libprt build (abtmp/ A/B copies) and compare it with
the CPU oracle pixel by pixel: fraction of identical pixels, RMSE, determinism over repeats.

    python tools/lib_vs_oracle.py --lib abtmp/libprt_x.so --res 128 --spp 4 --depth 4 --reps 3
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)
    from ab_builds import load
    from oracle import oracle as O
    from pyrenderer_amd import _native as N
    from pyrenderer_amd import scenes
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    N.lib()
    N._lib = load(a.lib)
    scene, camera = read_file(scenes.CORNELL)
    flat = flatten_scene(scene)
    cam = camera.convert_to_taichi_camera().packed()
    ds = DeviceScene(flat, 0)
    W = H = a.res
    ids = interleaved_tiles(W, H, 64)
    osc = O.OracleScene.from_flat(flat)
    ref = osc.render(cam, W, H, a.spp, a.depth, seed=a.seed)
    outs = []
    for _ in range(a.reps):
        out, _ = ds.render_tiles(cam, W, H, 64, 64, ids, a.spp, a.depth, a.seed, 0)
        from pyrenderer_amd.device_scene import unpack_tiles
        fr = np.zeros((W, H, 3), np.float32)
        unpack_tiles(out.reshape(-1, 3), W, H, 64, 64, ids, fr)
        outs.append(fr)   # per-pixel sums, like the oracle's render()
    same = [float(np.all(o == ref, axis=-1).mean()) for o in outs]
    rmse = [float(np.sqrt((((o.astype(np.float64) - ref) / a.spp) ** 2).mean())) for o in outs]
    det = all(np.array_equal(outs[0], o) for o in outs[1:])
    print(json.dumps({"lib": a.lib, "identical_pixels": same, "rmse": rmse, "deterministic": det,
                      "mean_gpu": float(outs[0].mean()), "mean_oracle": float(ref.mean())}), flush=True)
    ds.close()


if __name__ == "__main__":
    main()
