"""Command-line renderer: the build's counterpart of the reference's render scripts
(main_taichi.py:15-127 — read_file, World, PathTracer, progressive render() passes with a
samples/s print, finish() tone map, out.png every 100 passes; main.py:107-125's
--samples flag), without the Taichi GUI.

    python -m pyrenderer_amd [scene.json] --samples 64 --depth 16 --out out.png
    python -m pyrenderer_amd --samples 256 --interval 32 --state acc.npz      # resumable
    python -m pyrenderer_amd --samples 64 --devices 0 1 2 3                   # tiles over 4 GPUs

Every sample runs through libprt's HIP path (core.tracing.render / Accumulator); there is
no CPU fallback.
"""
import argparse
import os
import time

import numpy as np

from .core.tracing import Accumulator, as_image, render_sums
from .io_utils.read_tungsten import read_file
from .tone_map import finish, reinhard_extended, save_hdr, to_uint8, write_png

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_SCENE = os.path.join(HERE, "media", "cornell-box", "scene.json")


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="python -m pyrenderer_amd", description=__doc__.split("\n\n")[0])
    ap.add_argument("scene", nargs="?", default=DEFAULT_SCENE, help="Tungsten scene.json (default: Cornell box)")
    ap.add_argument("--samples", type=int, default=64, help="samples per pixel (main_taichi.py:29)")
    ap.add_argument("--depth", type=int, default=16, help="path depth (main_taichi.py:37)")
    ap.add_argument("--resolution", type=int, nargs=2, metavar=("W", "H"), help="override camera.resolution")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--devices", type=int, nargs="+", default=[0], help="GPUs of this process (tiles shard over them)")
    ap.add_argument("--nee", choices=["reference", "mis"], default="reference",
                    help="direct lighting: sample_direct_lighting (reference) or sample_direct_lighting2 (MIS)")
    ap.add_argument("--interval", type=int, default=0,
                    help="progressive passes of this many spp with a samples/s line each (one device; 0 = one pass)")
    ap.add_argument("--state", help="progressive accumulation file: resumed when it exists, saved after every pass")
    ap.add_argument("--tonemap", choices=["sqrt", "reinhard"], default="sqrt",
                    help="finish() = sqrt(pixels/samples) (main_taichi.py:61-64) or finishing_tonemap (:67-78)")
    ap.add_argument("--out", default="out.png", help="PNG path ('' = no image)")
    ap.add_argument("--hdr", metavar="DIR",
                    help="also save the reference's HDR pair (main_taichi.py:120-123) into DIR: hdr.npy = the "
                         "radiance sums (W, H, 3) [x][y], spp.npy = the per-pixel sample counts (W, H); "
                         "the reference's tone_map.py reads exactly these")
    args = ap.parse_args(argv)
    if args.hdr and args.hdr.lower().endswith(".npy"):
        # rounds <= 4 took a .npy FILE here; a directory named out.npy would silently replace it
        ap.error(f"--hdr takes a directory (hdr.npy and spp.npy are written into it), not a .npy file: {args.hdr}")
    return args


def _write(args, sums, samples, mean):
    if args.hdr:
        save_hdr(args.hdr, sums, samples)
    if args.out:
        img = finish(mean) if args.tonemap == "sqrt" else reinhard_extended(mean)
        write_png(args.out, to_uint8(as_image(img)))


def main(argv=None):
    args = parse(argv)
    scene, camera = read_file(args.scene)
    W, H = args.resolution if args.resolution else camera.resolution
    t0 = time.perf_counter()
    if args.interval > 0 or args.state:
        if len(args.devices) != 1:
            raise SystemExit("progressive rendering (--interval/--state) runs on one device")
        state = Accumulator.state_path(args.state) if args.state else None
        if state and os.path.exists(state):
            acc = Accumulator.load(state, scene, camera, device=args.devices[0])
            # the saved estimator settings win; refuse a command line that asks for others
            given = {"depth": args.depth, "seed": args.seed, "resolution": (W, H),
                     "nee": args.nee}
            saved = {"depth": acc.depth, "seed": acc.seed, "resolution": (acc.W, acc.H),
                     "nee": "mis" if acc.flags else "reference"}
            clash = [f"--{k} {given[k]} (saved: {saved[k]})" for k in given if given[k] != saved[k]]
            if clash:
                raise SystemExit(f"{state} was rendered with other settings: " + ", ".join(clash))
            print(f"resumed {state}: {acc.samples} spp")
        else:
            acc = Accumulator(scene, camera, depth=args.depth, seed=args.seed, resolution=(W, H),
                              device=args.devices[0], nee=args.nee)
        step = args.interval if args.interval > 0 else args.samples
        while acc.samples < args.samples:
            n = min(step, args.samples - acc.samples)
            t = time.perf_counter()
            acc.add(n)
            dt = time.perf_counter() - t
            print(f"{n / dt:.2f} samples/s ({acc.samples} spp, {W * H * n / dt / 1e6:.1f} Msamples/s)", flush=True)
            if state:
                acc.save(state)
        sums, samples, mean = acc.sums(), acc.samples, acc.mean()
        W, H = acc.W, acc.H
    else:
        sums = render_sums(scene, camera, spp=args.samples, depth=args.depth, seed=args.seed, resolution=(W, H),
                           devices=tuple(args.devices), nee=args.nee)
        samples = max(args.samples, 0)
        # render()'s mean, bit for bit: pixels / samples (main_taichi.py:61-64)
        mean = sums / np.float32(samples) if samples else np.zeros_like(sums)
    dt = time.perf_counter() - t0
    _write(args, sums, samples, mean)
    print(f"{W}x{H} x {args.samples} spp, depth {args.depth}: {dt:.2f} s "
          f"({W * H * args.samples / dt / 1e6:.1f} Msamples/s incl. scene build), mean RGB {mean.mean(axis=(0, 1))}")
    return mean


if __name__ == "__main__":
    main()
