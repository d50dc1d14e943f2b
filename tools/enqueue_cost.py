"""Host cost of enqueuing one frame (prt_render_tiles_device) against the device time of
that frame, for a small and a large workload: is the path launch-bound anywhere?

    python tools/enqueue_cost.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    scene, cam = bench.load_scene("cornell")
    flat = flatten_scene(scene)
    c = cam.convert_to_taichi_camera().packed()
    ds = DeviceScene(flat, 0)
    for res, spp, depth in [(128, 4, 4), (512, 64, 8)]:
        ids = interleaved_tiles(res, res, 64)
        buf = torch.zeros(len(ids) * 64 * 64 * 3, dtype=torch.float32, device="cuda:0")
        s = torch.cuda.current_stream()
        n = 200 if res == 128 else 20
        for _ in range(5):
            ds.render_tiles_device(c, res, res, 64, 64, ids, spp, depth, buf.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            ds.render_tiles_device(c, res, res, 64, 64, ids, spp, depth, buf.data_ptr(), s.cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"res": res, "spp": spp, "depth": depth, "frames": n,
                          "host_enqueue_us_per_frame": round((t1 - t0) / n * 1e6, 1),
                          "wall_us_per_frame_one_stream": round((t2 - t0) / n * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
