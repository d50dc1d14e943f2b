"""A/B the trace-kernel variants on one device, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Checks every variant's image is
bit-identical, prints per-variant median/min trace-kernel ms and Msamples/s.

    python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 5 --variants 1 2 3
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def vflags(v):
    """'7' -> variant 7's flag bits."""
    return int(v) << 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", nargs="+", default=["1", "2", "3"],
                    help="kernel variant numbers")
    ap.add_argument("--scene", default="cornell", help="cornell | cubes | soup:N (random triangle soup of N tris in the box)")
    a = ap.parse_args()
    from pyrenderer_amd._native import PRT_FLAG_TIME
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(os.path.join(ROOT, "pyrenderer_amd", "media", "cornell-box", "scene.json"))
    flat = flatten_scene(scene)
    if a.scene == "specular":
        from pyrenderer_amd.scenes import CORNELL_SPECULAR
        scene, cam = read_file(CORNELL_SPECULAR)
        flat = flatten_scene(scene)
    if a.scene == "cubes":
        from pyrenderer_amd.scenes import instanced_cubes
        scene, cam = instanced_cubes()
        flat = flatten_scene(scene)
    if a.scene.startswith("soup:"):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_gpu_parity import _soup_scene
        flat = _soup_scene((scene, cam, flat), int(a.scene.split(":")[1]), 9)
    ds = DeviceScene(flat, 0)
    c = cam.convert_to_taichi_camera().packed()
    W = H = a.res
    ids = interleaved_tiles(W, H, 64)
    res = {v: [] for v in a.variants}
    ref = None
    for r in range(a.rounds + 1):
        for v in a.variants:
            flags = PRT_FLAG_TIME | vflags(v)
            t0 = time.perf_counter()
            out, _ = ds.render_tiles(c, W, H, 64, 64, ids, a.spp, a.depth, 0, flags)
            wall = time.perf_counter() - t0
            ms, n = ds.kernel_timing()
            if ref is None:
                ref = out
            same = bool(np.array_equal(out, ref))
            if r > 0:  # round 0 = warm-up
                res[v].append((ms, wall * 1e3, same))
    samples = W * H * a.spp
    from pyrenderer_amd._native import PRT_FLAG_STATS
    for v in a.variants:
        ds.render_tiles(c, W, H, 64, 64, ids, a.spp, a.depth, 0, PRT_FLAG_STATS | vflags(v))
        dg = ds.diag_words(22).astype(np.float64)   # 17..21: ext / shadow iteration clocks, counts, lanes
        tot = dg[4] + dg[5] + dg[6]
        if v.rstrip("np") in ("7", "8", "9", "10"):
            # trace_kernel_pool's diag words 17..20: wave E iterations, wave S iterations, lanes of the
            # S iterations, shadow rays answered by the light-triangle test
            print(json.dumps({"variant": v, "pool": {
                "e_wave_iters": int(dg[17]), "s_wave_iters": int(dg[18]),
                "lanes_per_s_iter": round(dg[19] / max(dg[18], 1), 2),
                "s_iters_per_e_iter": round(dg[18] / max(dg[17], 1), 3),
                "shadow_queries": int(dg[3]), "answered_by_light_test": int(dg[20]),
                "nodes_per_sample": round(dg[0] / samples, 2), "tris_per_sample": round(dg[1] / samples, 2),
                "max_stack": int(dg[13])}}), flush=True)
            continue
        print(json.dumps({"variant": v, "diag": {"refill_frac": round(dg[4] / tot, 3), "trav_frac": round(dg[5] / tot, 3),
                                                 "shade_frac": round(dg[6] / tot, 3), "wave_iters": int(dg[7]),
                                                 "lanes_per_iter": round(dg[8] / max(dg[7], 1), 2),
                                                 "nodes_per_sample": round(dg[0] / samples, 2),
                                                 "tris_per_sample": round(dg[1] / samples, 2),
                                                 "inner_simd_eff": round(dg[11] / max(dg[9] * 64, 1), 3),
                                                 "leaf_simd_eff": round(dg[12] / max(dg[10] * 64, 1), 3),
                                                 "wave_inner_trips_per_iter": round(dg[9] / max(dg[7], 1), 2),
                                                 "wave_leaf_trips_per_iter": round(dg[10] / max(dg[7], 1), 2),
                                                 "wave_tri_trips_per_iter": round(dg[15] / max(dg[7], 1), 2),
                                                 "max_stack": int(dg[13]),
                                                 "max_nodes_one_query": int(dg[16]),
                                                 "shadow_iter_time_frac": round(dg[18] / max(dg[17] + dg[18], 1), 3),
                                                 "ext_iters": int(dg[19]), "shadow_iters": int(dg[20]),
                                                 "lanes_per_shadow_iter": round(dg[21] / max(dg[20], 1), 2),
                                                 "lanes_per_ext_iter": round((dg[8] - dg[21]) / max(dg[19], 1), 2)}}),
              flush=True)
    for v, rows in res.items():
        ms = np.array([x[0] for x in rows])
        wall = np.array([x[1] for x in rows])
        print(json.dumps({"variant": v, "kernel_ms_median": round(float(np.median(ms)), 3),
                          "wall_ms_median": round(float(np.median(wall)), 3),
                          "kernel_ms_min": round(float(ms.min()), 3),
                          "msamples_s": round(samples / np.median(ms) / 1e3, 1),
                          "identical_to_first": all(x[2] for x in rows), "scene": a.scene,
                          "bvh_depth": ds.bvh_depth, "nodes": ds.n_nodes}), flush=True)


if __name__ == "__main__":
    main()
