"""Shape of a persistent trace launch in time: every wave's start / end real-time stamp
(s_memrealtime, 100 MHz) and the work items it took, recorded by the kernel when
PRT_WAVE_CLOCK names a file (diagnostic read-back after each trace launch).

    python tools/wave_clock.py --config 4 [--reps 2]

Prints one JSON line per launch: span, when the first / median / last wave ended, the
fraction of the span with fewer than 50 % / 10 % of the waves still running (the drain),
and items per wave (load balance of the work queue).
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarise(rec):
    """rec: (n_waves, 3) u64 (start, end, items) of one launch -> dict (times in us)."""
    rec = rec[rec[:, 1] > 0]
    t0 = rec[:, 0].min()
    st = (rec[:, 0] - t0) / 100.0
    en = (rec[:, 1] - t0) / 100.0
    span = en.max()
    ts = np.linspace(0.0, span, 2001)
    alive = (st[None, :] <= ts[:, None]) & (en[None, :] > ts[:, None])
    frac = alive.mean(axis=1)
    dt = span / 2000.0
    items = rec[:, 2].astype(np.float64)
    return {"waves": int(rec.shape[0]), "span_us": round(float(span), 1),
            "start_spread_us": round(float(st.max()), 1),
            "start_pct_us": [round(float(np.percentile(st, q)), 1) for q in (25, 50, 57, 60, 75, 90)],
            "end_first_us": round(float(en.min()), 1), "end_p10_us": round(float(np.percentile(en, 10)), 1),
            "end_median_us": round(float(np.median(en)), 1), "end_p90_us": round(float(np.percentile(en, 90)), 1),
            "us_below_50pct_waves": round(float((frac[1:] < 0.5).sum() * dt), 1),
            "us_below_10pct_waves": round(float((frac[1:] < 0.1).sum() * dt), 1),
            "items_per_wave": {"mean": round(float(items.mean()), 1), "min": int(items.min()), "max": int(items.max())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--spp", type=int, default=None, help="override the config's samples per pixel")
    a = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(), "wave_clock.bin")
    os.environ["PRT_WAVE_CLOCK"] = path
    import bench
    from pyrenderer_amd._native import PRT_FLAG_TIME
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    cfg = bench.CONFIGS[a.config]
    scene, camera = bench.load_scene(cfg["scene"])
    ds = DeviceScene(flatten_scene(scene), 0)
    cam = camera.convert_to_taichi_camera().packed()
    W = H = cfg["res"]
    ids = interleaved_tiles(W, H, 64)
    waves = ds.blocks_per_cu * ds.cus * 4
    for rep in range(a.reps):
        if os.path.exists(path):
            os.remove(path)
        ds.render_tiles(cam, W, H, 64, 64, ids, a.spp or cfg["spp"], cfg["depth"], 0, PRT_FLAG_TIME | (a.variant << 8))
        ms, n = ds.kernel_timing()
        raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 3)
        per = raw.shape[0] // max(n, 1)
        for k in range(n):
            s = summarise(raw[k * per:(k + 1) * per])
            print(json.dumps({"config": a.config, "rep": rep, "launch": k, "kernel_ms_events": round(ms / n, 3),
                              "grid_waves": waves, **s}), flush=True)


if __name__ == "__main__":
    main()
