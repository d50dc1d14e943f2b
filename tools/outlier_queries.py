import os, sys, json, numpy as np
sys.path.insert(0, os.getcwd())
import bench
from pyrenderer_amd._native import PRT_FLAG_STATS
from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
from pyrenderer_amd.flatten import flatten_scene
cfg = bench.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 4]
scene, camera = bench.load_scene(cfg["scene"])
flat = flatten_scene(scene)
ds = DeviceScene(flat, 0)
cam = camera.convert_to_taichi_camera().packed()
ids = interleaved_tiles(cfg["res"], cfg["res"], 64)
ds.render_tiles(cam, cfg["res"], cfg["res"], 64, 64, ids, cfg["spp"], cfg["depth"], 0, PRT_FLAG_STATS)
w = ds.diag_words(24 + 128)
print("max_q", int(w[16]), "n_outliers", int(w[23]))
for k in range(min(16, int(w[23]))):
    r = w[24 + 8 * k: 32 + 8 * k]
    f = np.array(r[:7], np.uint64).astype(np.uint32).view(np.float32)
    print(json.dumps({"o": f[:3].tolist(), "d": f[3:6].tolist(), "tmax": float(f[6]), "qtype": int(r[7] >> 32), "nodes": int(r[7] & 0xffffffff)}))
