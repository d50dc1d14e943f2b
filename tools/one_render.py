"""Render one bench configuration a few times with a chosen kernel variant, for
profiling under rocprofv3 (one process, nothing else on the device):

    rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU ... -d OUT -o p --output-format csv \
        -- python tools/one_render.py --config 2 --variant 11 --reps 2
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--variant", type=int, default=0, help="0 = library default")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import bench
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    cfg = bench.CONFIGS[a.config]
    from pyrenderer_amd.flatten import flatten_scene
    scene, camera = bench.load_scene(cfg["scene"])
    flat = flatten_scene(scene)
    cam = camera.convert_to_taichi_camera().packed()
    ds = DeviceScene(flat, 0)
    W = H = cfg["res"]
    ids = interleaved_tiles(W, H, 64)
    for _ in range(a.reps):
        ds.render_tiles(cam, W, H, 64, 64, ids, cfg["spp"], cfg["depth"], 0, a.variant << 8)
    print("rendered", a.config, a.variant, a.reps)


if __name__ == "__main__":
    main()
