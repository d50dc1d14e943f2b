"""Build-defined benchmark scenes (BASELINE.json configs 3-5).

config 3: media/cornell-box/scene_specular.json (metal tall box, dielectric short box,
          dielectric sphere).
config 4: `instanced_cubes()` — media/cube.obj (12 triangles) instanced on a jittered 3-D grid
          inside the Cornell box (scale 0.01–0.03, rng seed 1234), walls and light kept:
          83 334 instances + 36 = 1 000 044 triangles.
"""
import os

import numpy as np

from .core.bsdf import BSDF
from .io_utils.read_tungsten import load_obj, read_file

MEDIA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "media")
CORNELL = os.path.join(MEDIA, "cornell-box", "scene.json")
CORNELL_SPECULAR = os.path.join(MEDIA, "cornell-box", "scene_specular.json")


class MeshBatch:
    """Many triangles under one BSDF, world-space already (vectorised TriangleMesh)."""
    type_name = "mesh"

    def __init__(self, vertices, faces, bsdf):
        from .mathematics.bbox import BBox
        self.id = -1
        self.vertices = np.asarray(vertices, np.float64)
        self.faces = np.asarray(faces, np.int64)
        self.bsdf = bsdf
        tri = self.vertices[self.faces]
        e1 = tri[:, 1] - tri[:, 0]
        e2 = tri[:, 2] - tri[:, 0]
        c = np.cross(e1, e2)
        n = np.sqrt(c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1] + c[:, 2] * c[:, 2])
        self.normal_vectors = (c / n[:, None]).astype(np.float32)   # Cube convention: +normalize(e1 x e2)
        self.bounds = BBox(None, None)
        self.bounds.from_vertices(self.vertices)
        self.center = self.bounds.center()

    @property
    def bounding_box(self):
        return self.bounds.min_coord, self.bounds.max_coord


def instanced_cubes(n_instances=83334, seed=1234, scale=(0.01, 0.03), albedo=(0.725, 0.71, 0.68)):
    """Config 4: Cornell box + n_instances jittered, scaled copies of media/cube.obj."""
    scene, cam = read_file(CORNELL)
    v, f = load_obj(os.path.join(MEDIA, "cube.obj"))
    rng = np.random.default_rng(seed)
    g = int(np.ceil(n_instances ** (1.0 / 3.0)))
    cells = np.stack(np.meshgrid(np.arange(g), np.arange(g), np.arange(g), indexing="ij"), -1).reshape(-1, 3)
    cells = cells[rng.permutation(cells.shape[0])[:n_instances]]
    lo = np.array([-0.95, 0.02, -0.95])
    hi = np.array([0.95, 1.90, 0.95])
    size = (hi - lo) / g
    s = rng.uniform(scale[0], scale[1], n_instances)
    origin = lo + (cells + rng.uniform(0.1, 0.9, (n_instances, 3))) * size - 0.5 * s[:, None]
    verts = (v[None, :, :] - 0.0) * s[:, None, None] + origin[:, None, :]          # cube.obj spans [0,1]^3
    faces = f[None, :, :] + (np.arange(n_instances) * v.shape[0])[:, None, None]
    mat = BSDF({"type": "lambert", "albedo": list(albedo)}).get_distribution()
    scene.add_primitive(MeshBatch(verts.reshape(-1, 3), faces.reshape(-1, 3), mat))
    return scene, cam
