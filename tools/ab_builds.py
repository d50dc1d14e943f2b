"""A/B two builds of libprt.so in ONE process (same device, same clocks): each library is
loaded with ctypes (RTLD_LOCAL, its own HIP module), gets its own scene, and the rounds
interleave device-resident frames of both; images must be identical.

    python tools/ab_builds.py --libs abtmp/libprt_a.so abtmp/libprt_b.so --config 2 --rounds 5
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    from pyrenderer_amd import _native as N
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in N.EXPORTS.items():
        if not hasattr(L, name):   # an older build: entry points added since are not used here
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--variant", type=int, default=0, help="trace-kernel variant for every library (0 = default)")
    ap.add_argument("--spp", type=int, default=0, help="samples per pixel instead of the config's (launch-size probes)")
    a = ap.parse_args()
    import torch

    import bench
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    N.lib()   # torch first, then the default library (one HIP runtime for all)
    cfg = dict(bench.CONFIGS[a.config])
    if a.spp > 0:
        cfg["spp"] = a.spp
    scene, camera = bench.load_scene(cfg["scene"])
    flat = flatten_scene(scene)
    cam = camera.convert_to_taichi_camera().packed()
    W = H = cfg["res"]
    ids = interleaved_tiles(W, H, 64)
    libs = [load(p) for p in a.libs]
    scenes = []
    for L in libs:
        N._lib = L
        scenes.append(DeviceScene(flat, 0))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    buf = torch.empty(len(ids) * 64 * 64 * 3, dtype=torch.float32, device=dev)
    res = [[] for _ in libs]
    ref = None
    for r in range(a.rounds + 1):
        for k, (L, ds) in enumerate(zip(libs, scenes)):
            N._lib = L
            # one untimed launch first: the device idled during the previous library's host-side
            # compare, and the first launch after an idle gap runs at a lower clock
            ds.render_tiles_device(cam, W, H, 64, 64, ids, cfg["spp"], cfg["depth"], buf.data_ptr(),
                                   stream.cuda_stream, flags=N.PRT_FLAG_TIME | (a.variant << 8))
            torch.cuda.synchronize(dev)
            ds.kernel_timing()
            for _ in range(a.launches):
                ds.render_tiles_device(cam, W, H, 64, 64, ids, cfg["spp"], cfg["depth"], buf.data_ptr(),
                                       stream.cuda_stream, flags=N.PRT_FLAG_TIME | (a.variant << 8))
            torch.cuda.synchronize(dev)
            ms, n = ds.kernel_timing()
            out = buf.cpu().numpy()
            if ref is None:
                ref = out
            if r > 0:
                res[k].append((ms / max(n, 1), bool(np.array_equal(out, ref))))
    samples = W * H * cfg["spp"]
    for p, rows in zip(a.libs, res):
        ms = np.array([x[0] for x in rows])
        print(json.dumps({"lib": p, "config": a.config, "kernel_ms_median": round(float(np.median(ms)), 4),
                          "kernel_ms_min": round(float(ms.min()), 4), "kernel_ms_all": [round(float(x), 4) for x in ms],
                          "msamples_s": round(samples / np.median(ms) / 1e3, 1),
                          "identical": all(x[1] for x in rows)}), flush=True)
    # each scene handle belongs to its own library: destroy it through that library
    for L, ds in zip(libs, scenes):
        N._lib = L
        ds.close()


if __name__ == "__main__":
    main()
