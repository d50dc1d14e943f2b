"""Path tracing entry points (reference: core/tracing.py:47-155, main_taichi.py:80-127).

`render(scene, camera, spp=..., depth=...)` is the build's `core.tracing.render()`
(named by BASELINE.json's north star; the reference has only the Taichi
`render()` closure of main_taichi.py:80-99).  It returns the MEAN linear
radiance per pixel — `pixels / samples` of main_taichi.py:61-64 before the
sqrt tone map — as float32 (W, H, 3) indexed [x][y] with y up, like the
reference's `pixels.to_numpy()`.  Every sample runs PathTracer.trace's
estimator in the HIP kernel (pyrenderer_amd/csrc/prt_kernels.hip).

`devices=(0, 1, ...)` shards 64x64 tiles across GPUs of this process
('latin' interleave, device_scene.tile_owner) through prt_render_multi, which
gathers the tile sums to the first device with one RCCL send/recv group; the
image is bit-identical for any device count since random numbers are keyed by
(seed, global pixel, sample).  For one process per GPU use
pyrenderer_amd.distributed (torch.distributed gather over RCCL/xGMI).

`Accumulator` is the progressive form of main_taichi.py:108-127 (render() once
per GUI frame, pixels += L, samples += 1, finish() of the running mean), with
save / load to resume an accumulation.
"""
import hashlib
import os

import numpy as np

from ..device_scene import interleaved_tiles, render_multi, unpack_tiles
from ..mathematics.intersection import World


class PathTracer:
    """Same constructor as the reference (core/tracing.py:47-50).  `trace` runs the reference's
    per-ray estimator for a batch of caller rays; `render_sums` / `render` run render()'s
    per-pixel sample loop (main_taichi.py:80-99) over the whole frame."""

    def __init__(self, world, depth, img_w, img_h):
        self.world = world
        self.depth = depth
        self.img_w = img_w
        self.img_h = img_h

    def trace(self, ro, rd, depth=None, x=None, y=None, *, seed=0, device=0, nee="reference"):
        """PathTracer.trace (core/tracing.py:116-155) on the GPU: the radiance of one path per ray,
        for one ray ((3,) arrays) or a batch ((n, 3) arrays), as float32 (3,) / (n, 3).

        depth defaults to the constructor's.  x, y are accepted for the reference's signature
        (its trace ignores them).  Ray i draws from the random stream keyed (seed, i, 0): the
        streams render() uses minus the two camera-jitter draws (include/prt.h prt_trace_rays)."""
        o = np.asarray(ro, np.float32)
        single = o.ndim == 1
        ds = self.world.device_scene(device)
        out = ds.trace_rays(o, rd, self.depth if depth is None else int(depth), seed=seed, flags=nee_flags(nee))
        return out[0] if single else out

    def render_sums(self, cam_packed, spp, seed=0, devices=(0,), tile=64, flags=0):
        """Per-pixel radiance SUMS over spp samples, (W, H, 3) [x][y]."""
        W, H = self.img_w, self.img_h
        devices = tuple(devices)
        if len(devices) > 1:
            return render_multi([self.world.device_scene(d) for d in devices], cam_packed, W, H, tile, spp,
                                self.depth, seed, flags)
        ds = self.world.device_scene(devices[0])
        ids = interleaved_tiles(W, H, tile)
        sums, _ = ds.render_tiles(cam_packed, W, H, tile, tile, ids, spp, self.depth, seed, flags)
        return unpack_tiles(sums, W, H, tile, tile, ids)

    def render(self, cam_packed, spp, seed=0, devices=(0,), tile=64, nee="reference"):
        if spp <= 0:
            return np.zeros((self.img_w, self.img_h, 3), np.float32)
        return self.render_sums(cam_packed, spp, seed, devices, tile, nee_flags(nee)) / np.float32(spp)


def nee_flags(nee):
    """Direct-lighting estimator: 'reference' = sample_direct_lighting, the one the
    reference's trace calls (core/tracing.py:92-108, :150-151); 'mis' = its unused MIS
    alternative sample_direct_lighting2 (core/tracing.py:57-90) in the same place."""
    from .._native import PRT_FLAG_MIS_NEE
    if nee == "reference":
        return 0
    if nee == "mis":
        return PRT_FLAG_MIS_NEE
    raise ValueError(f"nee must be 'reference' or 'mis', not {nee!r}")


def build_world(scene, devices=(0,)):
    world = World()
    for p in scene.primitives:
        world.add(p)
    return world.commit(devices)


def render(scene, camera, *, spp, depth, seed=0, resolution=None, devices=(0,), tile=64, world=None,
           nee="reference"):
    """Mean linear radiance (W, H, 3) float32, [x][y], y up.

    nee: 'reference' (sample_direct_lighting, what the reference's trace runs) or 'mis'
    (the reference's unused MIS estimator sample_direct_lighting2, as an optional variant).

    resolution: (W, H) override of camera.resolution (the aspect ratio still
    comes from camera.resolution, as convert_to_taichi_camera() does).
    """
    W, H = resolution if resolution is not None else camera.resolution
    world = world or build_world(scene, devices)
    tracer = PathTracer(world, depth, int(W), int(H))
    return tracer.render(camera.convert_to_taichi_camera().packed(), spp, seed, devices, tile, nee)


def render_sums(scene, camera, *, spp, depth, seed=0, resolution=None, devices=(0,), tile=64, world=None,
                nee="reference"):
    """Per-pixel radiance SUMS (W, H, 3) float32 [x][y] over spp samples — the reference's `pixels`
    field after spp render() passes (main_taichi.py:97); render() returns these / spp."""
    W, H = resolution if resolution is not None else camera.resolution
    world = world or build_world(scene, devices)
    tracer = PathTracer(world, depth, int(W), int(H))
    if spp <= 0:
        return np.zeros((int(W), int(H), 3), np.float32)
    return tracer.render_sums(camera.convert_to_taichi_camera().packed(), spp, seed, devices, tile, nee_flags(nee))


class Accumulator:
    """Progressive rendering on one device (main_taichi.py:108-127).

    `add(spp)` renders the next `spp` samples of every pixel and adds them in sample
    order onto the running per-pixel sums, so any split of N samples over add() calls
    leaves the sums bit-identical to `render(spp=N)` * N.  `mean()` is
    pixels / samples (main_taichi.py:61-64, before the sqrt tone map).  `save(path)` /
    `Accumulator.load(path, scene, camera)` resume an accumulation (.npz: sums, sample
    count, seed, depth, resolution, tile, estimator flags, the packed camera and a
    fingerprint of the flattened scene — load() refuses a different camera or scene,
    whose samples would otherwise be averaged into the same image).
    """

    def __init__(self, scene, camera, *, depth, seed=0, resolution=None, device=0, tile=64, world=None,
                 nee="reference"):
        W, H = resolution if resolution is not None else camera.resolution
        self.W, self.H, self.depth, self.seed, self.tile = int(W), int(H), int(depth), int(seed), int(tile)
        self.device = device
        self.world = world or build_world(scene, (device,))
        self.cam = camera.convert_to_taichi_camera().packed()
        self.ids = interleaved_tiles(self.W, self.H, self.tile)
        self.slots = np.zeros((self.ids.shape[0] * self.tile * self.tile, 3), np.float32)
        self.samples = 0
        self.flags = nee_flags(nee)

    def add(self, spp=1):
        """Render samples [samples, samples + spp) of every pixel onto the sums."""
        if spp < 0:
            raise ValueError("spp must be >= 0")
        ds = self.world.device_scene(self.device)
        ds.render_tiles_accumulate(self.cam, self.W, self.H, self.tile, self.tile, self.ids, self.samples, spp,
                                   self.depth, self.slots, self.seed, self.flags)
        self.samples += spp
        return self

    def sums(self):
        """Per-pixel radiance sums (W, H, 3) [x][y] — the reference's `pixels` field."""
        return unpack_tiles(self.slots, self.W, self.H, self.tile, self.tile, self.ids)

    def mean(self):
        if self.samples == 0:
            return np.zeros((self.W, self.H, 3), np.float32)
        return self.sums() / np.float32(self.samples)

    def state(self):
        return dict(slots=self.slots, samples=np.int64(self.samples), seed=np.int64(self.seed),
                    depth=np.int64(self.depth), resolution=np.array([self.W, self.H], np.int64),
                    tile=np.int64(self.tile), flags=np.int64(self.flags), camera=self.cam,
                    scene_sha=np.array(scene_fingerprint(self.world.flat)))

    @staticmethod
    def state_path(path):
        """np.savez appends '.npz' to a path without it: save and load use the same name."""
        path = os.fspath(path)
        return path if path.endswith(".npz") else path + ".npz"

    def save(self, path):
        np.savez(self.state_path(path), **self.state())

    @classmethod
    def load(cls, path, scene, camera, device=0, world=None):
        z = np.load(cls.state_path(path), allow_pickle=False)
        W, H = (int(v) for v in z["resolution"])
        mis = "flags" in z.files and int(z["flags"]) & nee_flags("mis")
        acc = cls(scene, camera, depth=int(z["depth"]), seed=int(z["seed"]), resolution=(W, H), device=device,
                  tile=int(z["tile"]), world=world, nee="mis" if mis else "reference")
        if z["slots"].shape != acc.slots.shape:
            raise ValueError("saved accumulation does not match the frame layout")
        if "camera" in z.files and not np.array_equal(z["camera"], acc.cam):
            raise ValueError("saved accumulation was rendered with a different camera")
        if "scene_sha" in z.files and str(z["scene_sha"]) != scene_fingerprint(acc.world.flat):
            raise ValueError("saved accumulation was rendered from a different scene")
        acc.slots[...] = z["slots"]
        acc.samples = int(z["samples"])
        return acc


def scene_fingerprint(flat):
    """SHA-256 (hex, 16 chars) of the flattened scene arrays the kernel renders."""
    h = hashlib.sha256()
    for k in ("tri_v", "tri_n", "tri_mat", "mat", "light_tri", "light_off", "direct_rgb", "sph", "sph_mat"):
        a = getattr(flat, k, None)
        if a is not None:
            a = np.ascontiguousarray(a)
            h.update(k.encode() + str(a.dtype).encode() + str(a.shape).encode() + a.tobytes())
    return h.hexdigest()[:16]


def as_image(radiance_xy):
    """[x][y] (y up) → [row][col] top row first, as main.py:55 writes images."""
    return np.ascontiguousarray(np.asarray(radiance_xy).transpose(1, 0, 2)[::-1])
