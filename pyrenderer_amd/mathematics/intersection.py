"""World: primitive registry + commit to the GPU
(reference: mathematics/intersection_taichi.py:188-233).

`World.add` keeps insertion order and the light list exactly like the
reference; `World.commit()` flattens the primitives (pyrenderer_amd/flatten.py),
builds the triangle BVH and uploads everything through prt_scene_create.
Intersection itself (`hit_all`) runs inside the HIP kernel.
"""
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
