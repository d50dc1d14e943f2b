"""A/B the scene-creation knobs (env PRT_SAH_CT, PRT_SAH_BINS, PRT_LEAF_MIN, PRT_MAX_LEAF,
PRT_LEAF_BREAK, PRT_RESUME_MIN) on one device: one scene per setting, interleaved timed
rounds of `--launches` device-resident frames each (HIP-event kernel time), counted work
per sample, and a check that every setting renders the identical image (closest hits do
not depend on the tree or the traversal schedule).

    python tools/bvh_knobs.py --config 2 --settings "" "PRT_SAH_CT=1" "PRT_MAX_LEAF=8,PRT_LEAF_MIN=1"
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KNOBS = ("PRT_SAH_CT", "PRT_SAH_BINS", "PRT_LEAF_MIN", "PRT_MAX_LEAF", "PRT_LEAF_BREAK", "PRT_LEAF_EXIT", "PRT_RESUME_MIN")


def apply(setting):
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--launches", type=int, default=5, help="timed frames per setting per round")
    ap.add_argument("--settings", nargs="+", default=[""])
    a = ap.parse_args()
    import bench
    from pyrenderer_amd._native import PRT_FLAG_STATS, PRT_FLAG_TIME
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    cfg = bench.CONFIGS[a.config]
    scene, camera = bench.load_scene(cfg["scene"])
    flat = flatten_scene(scene)
    cam = camera.convert_to_taichi_camera().packed()
    W = H = cfg["res"]
    ids = interleaved_tiles(W, H, 64)
    samples = W * H * cfg["spp"]
    scenes, res, ref = {}, {}, None
    for s in a.settings:
        apply(s)
        scenes[s] = DeviceScene(flat, 0)
        res[s] = []
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    buf = torch.empty(len(ids) * 64 * 64 * 3, dtype=torch.float32, device=dev)
    for r in range(a.rounds + 1):
        for s in a.settings:
            apply(s)
            scenes[s].kernel_timing()
            for _ in range(a.launches):
                scenes[s].render_tiles_device(cam, W, H, 64, 64, ids, cfg["spp"], cfg["depth"], buf.data_ptr(),
                                              stream.cuda_stream, flags=PRT_FLAG_TIME | (a.variant << 8))
            torch.cuda.synchronize(dev)
            ms, n = scenes[s].kernel_timing()
            out = buf.cpu().numpy()
            if ref is None:
                ref = out
            if r > 0:
                res[s].append((ms / max(n, 1), bool(np.array_equal(out, ref))))
    for s in a.settings:
        apply(s)
        ds = scenes[s]
        ds.render_tiles(cam, W, H, 64, 64, ids, cfg["spp"], cfg["depth"], 0, PRT_FLAG_STATS | (a.variant << 8))
        st = ds.last_stats().astype(np.float64)
        ms = np.array([x[0] for x in res[s]])
        print(json.dumps({"setting": s or "default", "config": a.config, "kernel_ms_median": round(float(np.median(ms)), 3),
                          "kernel_ms_min": round(float(ms.min()), 3),
                          "msamples_s": round(samples / np.median(ms) / 1e3, 1),
                          "nodes_per_sample": round(st[0] / samples, 2), "tris_per_sample": round(st[1] / samples, 2),
                          "bvh_nodes": ds.n_nodes, "bvh_depth": ds.bvh_depth, "kernel": ds.kernel_info(),
                          "identical": all(x[1] for x in res[s])}), flush=True)
        ds.close()


if __name__ == "__main__":
    main()
