"""World: primitive registry + commit to the GPU
(reference: mathematics/intersection_taichi.py:188-291).

`World.add` keeps insertion order and the light list exactly like the
reference; `World.commit()` flattens the primitives (pyrenderer_amd/flatten.py),
builds the triangle BVH and uploads everything through prt_scene_create.
`World.hit_all` is the reference's closest-hit query for a batch of rays, run on
the GPU through prt_hit_all (the path tracer itself calls it inside the HIP kernel).
"""
import numpy as np

from ..device_scene import DeviceScene
from ..flatten import flatten_scene


class _PrimList:
    def __init__(self, prims):
        self.primitives = prims


class World:
    def __init__(self):
        self.primitives = []
        self.lights = []
        self.device_scenes = {}

    def add(self, prim):
        prim.id = len(self.primitives)
        self.primitives.append(prim)
        if prim.bsdf.emitting_light:
            self.lights.append(prim)

    def commit(self, devices=(0,)):
        """Should be called after all objects are added; uploads to every device."""
        assert len(self.lights) > 0, "There is no lights!!!"
        self.flat = flatten_scene(_PrimList(self.primitives))
        for d in devices:
            if d not in self.device_scenes:
                self.device_scenes[d] = DeviceScene(self.flat, d)
        return self

    def device_scene(self, device=0):
        if device not in self.device_scenes:
            self.commit(devices=(device,))
        return self.device_scenes[device]

    def hit_all(self, ray_origin, ray_direction, t_min, closest_so_far, *, seed=0, device=0):
        """World.hit_all (intersection_taichi.py:238-291) for one ray ((3,) arrays) or a batch
        ((n, 3) arrays; t_min / closest_so_far scalars or (n,) arrays), on the GPU.

        Returns the reference's 8-tuple (hit_anything, closest_so_far, p, normal, emissive,
        attenuation, scattered_dir, pdf): closest hit of the strict t_min < t < closest_so_far
        test (closest_so_far is returned unchanged on a miss), p = o + t d, the face normal
        flipped toward the ray for two-sided BSDFs, the BSDF's emitting flag and evaluate(), and
        the BSDF scatter at the hit (cosine-hemisphere draw in the normal frame, pdf = |n.wi|/pi).
        The reference draws the scatter from Taichi's stateful RNG inside hit_all; here ray i
        draws from the stream keyed (seed, i, 0) (include/prt.h prt_hit_all)."""
        o = np.asarray(ray_origin, np.float32)
        single = o.ndim == 1
        out = self.device_scene(device).hit_all(o, ray_direction, t_min, closest_so_far, seed=seed)
        res = (out[:, 0] > 0, out[:, 1].copy(), out[:, 2:5].copy(), out[:, 5:8].copy(),
               out[:, 8].astype(np.int32), out[:, 9:12].copy(), out[:, 12:15].copy(), out[:, 15].copy())
        if single:
            return tuple(r[0] for r in res)
        return res
