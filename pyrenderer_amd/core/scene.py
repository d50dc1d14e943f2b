"""Scene container (reference: core/scene.py:11-46).

Holds primitives and lights in insertion order and the concatenated
vertices/faces, as the reference does.  The CPU `hit`/BVH helpers of the
reference's NumPy debug stack are out of scope.
"""
import random

import numpy as np


class Scene:
    def __init__(self):
        self.primitives = []
        self.lights = []
        self.vertices = None
        self.faces = None

    def add_primitive(self, prim):
        self.primitives.append(prim)
        if prim.bsdf.emitting_light:
            self.lights.append(prim)
        if not hasattr(prim, "faces"):
            return
        if self.vertices is None:
            self.vertices = prim.vertices
            self.faces = prim.faces
        else:
            increment = self.vertices.shape[0]
            self.vertices = np.vstack([self.vertices, prim.vertices])
            self.faces = np.vstack([self.faces, prim.faces + increment])

    def sample_light(self):
        """A point on a random light (core/scene.py:23-28: random.choice(lights).sample_a_point()).
        Host-side debug API of the reference's NumPy stack; the renderer samples lights on the GPU."""
        if len(self.lights) > 0:
            return random.choice(self.lights).sample_a_point()
        print("[WARNING] no lights found")
        return None
