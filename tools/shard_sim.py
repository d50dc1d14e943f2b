"""Predict multi-GPU tile balance on ONE GPU: render, one rank at a time, exactly the
tiles rank r of N would own (device_scene.tile_owner) and time it.  The slowest
rank's time bounds the N-GPU step (plus the gather); T1 / (N * max_r T_r) is the
balance-limited strong-scaling efficiency.

    python tools/shard_sim.py [--config 2] [--tiles 64,32] [--schemes mod,latin] [--worlds 2,4,8]

Prints one JSON line per (tile, scheme, world).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--tiles", default="64,32")
    ap.add_argument("--schemes", default="mod,latin")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--streams", type=int, default=1, help="frames in flight, as bench.py --streams")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--frames", type=int, default=1,
                    help="frames per render call (prt_render_frames_device, bench.py --frames-per-launch), "
                         "gathered by one collective; --steps is then a multiple of it")
    ap.add_argument("--proxy", default="none", choices=("none", "stream", "stream-hp", "stream-nowait", "inline"),
                    help="after each frame, a copy of its tile buffer standing in for the RCCL gather: 'stream' on "
                         "one extra stream, ordered as torch's ProcessGroupNCCL orders a collective (the extra stream "
                         "waits for the frame, the frame's stream waits for the copy); 'inline' on the frame's own "
                         "stream (a gather enqueued on the render stream); 'stream-hp' as 'stream' on a high-priority "
                         "stream (TORCH_NCCL_HIGH_PRIORITY=1); 'stream-nowait' as 'stream' without the frame stream's "
                         "wait (timing only)")
    ap.add_argument("--no-null-stream", action="store_true",
                    help="render every frame on a created stream (default: the first on torch's current stream)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles, max_tiles_per_rank
    from pyrenderer_amd.flatten import flatten_scene

    cfg = bench.CONFIGS[a.config]
    scene, camera = bench.load_scene(cfg["scene"])
    flat = flatten_scene(scene)
    cam = camera.convert_to_taichi_camera().packed()
    ds = DeviceScene(flat, 0)
    W = H = cfg["res"]
    dev = torch.device("cuda", 0)
    streams = ([] if a.no_null_stream else [torch.cuda.current_stream(dev)])
    streams += [torch.cuda.Stream(dev) for _ in range(a.streams - len(streams))]
    coll = (torch.cuda.Stream(dev, priority=-1) if a.proxy == "stream-hp" else
            torch.cuda.Stream(dev) if a.proxy in ("stream", "stream-nowait") else None)

    def gather_proxy(buf, st, dst):
        if a.proxy == "inline":
            with torch.cuda.stream(st):
                dst.copy_(buf)
        if coll is None:
            return
        ev = torch.cuda.Event()
        ev.record(st)
        coll.wait_event(ev)
        with torch.cuda.stream(coll):
            dst.copy_(buf)
        if a.proxy != "stream-nowait":
            done = torch.cuda.Event()
            done.record(coll)
            st.wait_event(done)

    F = max(1, a.frames)

    def render(ids, tile, buf, st, flags):
        if F == 1:
            ds.render_tiles_device(cam, W, H, tile, tile, ids, cfg["spp"], cfg["depth"], buf.data_ptr(), st.cuda_stream,
                                   flags=flags | (a.variant << 8))
        else:
            ds.render_frames_device(cam, W, H, tile, tile, ids, cfg["spp"], cfg["depth"], F, buf.data_ptr(),
                                    st.cuda_stream, flags=flags | (a.variant << 8))

    def time_tiles(tile, ids):
        n = max(len(ids), 1) * tile * tile * 3
        bufs = [torch.empty(F * n, dtype=torch.float32, device=dev) for _ in streams]
        dst = torch.empty(F * n, dtype=torch.float32, device=dev)
        for b, st in zip(bufs, streams):
            render(ids, tile, b, st, 0)
        torch.cuda.synchronize(dev)
        ds.kernel_timing()
        groups = max(1, a.steps // F)
        t0 = time.perf_counter()
        for i in range(groups):
            k = i % len(streams)
            render(ids, tile, bufs[k], streams[k], N.PRT_FLAG_TIME)
            gather_proxy(bufs[k], streams[k], dst)   # one gather per group of F frames (bench.py)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) * 1e3 / (groups * F)
        kms, launches = ds.kernel_timing()
        return wall, kms / max(launches, 1) / F

    for tile in [int(t) for t in a.tiles.split(",")]:
        t1_wall, t1_k = time_tiles(tile, interleaved_tiles(W, H, tile))
        print(json.dumps({"tile": tile, "world": 1, "streams": a.streams, "frames": F, "proxy": a.proxy, "variant": a.variant, "wall_ms": round(t1_wall, 4), "kernel_ms": round(t1_k, 4)}),
              flush=True)
        for scheme in a.schemes.split(","):
            for world in [int(w) for w in a.worlds.split(",")]:
                walls, kerns = [], []
                for r in range(world):
                    w, k = time_tiles(tile, interleaved_tiles(W, H, tile, r, world, scheme))
                    walls.append(w)
                    kerns.append(k)
                print(json.dumps({
                    "tile": tile, "scheme": scheme, "world": world, "streams": a.streams, "frames": F, "proxy": a.proxy,
                    "max_tiles": max_tiles_per_rank(W, H, tile, world, scheme),
                    "wall_ms": [round(x, 4) for x in walls], "kernel_ms": [round(x, 4) for x in kerns],
                    "kernel_max_over_mean": round(max(kerns) / (sum(kerns) / world), 4),
                    "eff_wall": round(t1_wall / (world * max(walls)), 4),
                    "eff_kernel": round(t1_k / (world * max(kerns)), 4)}), flush=True)
    ds.close()


if __name__ == "__main__":
    main()
