"""Host-side primitives (reference: mathematics/shapes.py:15-243).

Only geometry set-up lives here — world-space vertices, faces, face normals,
bounds — with the reference's attribute names.  Intersection and sampling
(`Quad.hit`, `Quad.sample_a_point`, ...) run in the HIP kernels behind the
C-ABI (pyrenderer_amd/csrc), fed by `FlatScene` (pyrenderer_amd/flatten.py).

Vertex transform = trimesh `apply_transform` (M @ [v,1]^T in float64); face
winding is reversed when det(M[:3,:3]) < 0.  Normals: Quad uses
-normalize(e1 x e2) (shapes.py:43-47), Cube +normalize(e1 x e2) (shapes.py:172-176),
computed in float64 and stored float32 as the reference's arrays are.
"""
import math
import random

import numpy as np

from .bbox import BBox

QUAD_VERTICES = np.array([[-0.5, 0, -0.5], [0.5, 0, -0.5], [0.5, 0, 0.5], [-0.5, 0, 0.5]], np.float64)
QUAD_FACES = np.array([[0, 1, 2], [2, 3, 0]], np.int64)

CUBE_VERTICES = np.array([
    [-0.5, -0.5, -0.5], [-0.5, -0.5, 0.5], [0.5, -0.5, 0.5], [0.5, -0.5, -0.5],
    [-0.5, 0.5, 0.5], [-0.5, 0.5, -0.5], [0.5, 0.5, -0.5], [0.5, 0.5, 0.5],
    [-0.5, 0.5, -0.5], [-0.5, -0.5, -0.5], [0.5, -0.5, -0.5], [0.5, 0.5, -0.5],
    [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [-0.5, -0.5, 0.5], [-0.5, 0.5, 0.5],
    [-0.5, 0.5, 0.5], [-0.5, -0.5, 0.5], [-0.5, -0.5, -0.5], [-0.5, 0.5, -0.5],
    [0.5, 0.5, -0.5], [0.5, -0.5, -0.5], [0.5, -0.5, 0.5], [0.5, 0.5, 0.5]], np.float64)
CUBE_FACES = np.array([[2, 1, 0], [0, 3, 2], [6, 5, 4], [4, 7, 6], [10, 9, 8], [8, 11, 10],
                       [14, 13, 12], [12, 15, 14], [18, 17, 16], [16, 19, 18], [22, 21, 20], [20, 23, 22]], np.int64)


def normalize_vector(v):
    """mathematics/vec3.py:14-18 (v / sqrt(v.v), Python float sqrt)."""
    n = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    return v / n


def apply_transform(vertices, faces, matrix):
    m = np.asarray(matrix, dtype=np.float64)
    pts = np.asarray(vertices, dtype=np.float64)
    homo = np.column_stack((pts, np.ones(len(pts))))
    out = np.ascontiguousarray(np.dot(m, homo.T).T[:, :3])
    if np.linalg.det(m[:3, :3]) < 0:
        faces = np.ascontiguousarray(faces[:, ::-1])
    return out, faces


class _MeshPrimitive:
    normal_sign = 1.0
    type_name = "mesh"

    def __init__(self, trans_mat, bsdf, vertices, faces):
        self.id = -1
        self.trans_mat = trans_mat
        self.bsdf = bsdf
        self.vertices, self.faces = apply_transform(vertices, faces, trans_mat)
        self.normal_vectors = np.zeros((self.faces.shape[0], 3), np.float32)
        for i in range(self.faces.shape[0]):
            tri = self.faces[i]
            e1 = self.vertices[tri[1]] - self.vertices[tri[0]]
            e2 = self.vertices[tri[2]] - self.vertices[tri[0]]
            self.normal_vectors[i] = self.normal_sign * normalize_vector(np.cross(e1, e2))
        self.bounds = BBox(None, None)
        self.bounds.from_vertices(self.vertices)
        self.center = self.bounds.center()

    @property
    def bounding_box(self):
        return self.bounds.min_coord, self.bounds.max_coord

    def sample_a_point(self, rng=random):
        """A uniform point on a random face (the reference's NumPy twin, shapes2.py:72-79, used by
        Scene.sample_light): face randint(0, F-1), u = sqrt(U), v = U, a = u(1-v), b = uv,
        a V0 + b V1 + (1-a-b) V2.  Host-side (debug API); the kernel's light sampling is
        World.sample_a_light's (shapes.py:62-71) on the GPU."""
        face_id = rng.randint(0, self.faces.shape[0] - 1)
        u = math.sqrt(rng.uniform(0, 1))
        v = rng.uniform(0, 1)
        a = u * (1 - v)
        b = u * v
        v0, v1, v2 = self.faces[face_id]
        return a * self.vertices[v0] + b * self.vertices[v1] + (1.0 - a - b) * self.vertices[v2]


class Quad(_MeshPrimitive):
    """Unit quad in the xz plane, 2 triangles (shapes.py:15-57)."""
    normal_sign = -1.0
    type_name = "quad"

    def __init__(self, trans_mat, bsdf):
        super().__init__(trans_mat, bsdf, QUAD_VERTICES, QUAD_FACES)


class Cube(_MeshPrimitive):
    """Unit cube, 24 vertices / 12 triangles (shapes.py:117-186)."""
    normal_sign = 1.0
    type_name = "cube"

    def __init__(self, trans_mat, bsdf):
        super().__init__(trans_mat, bsdf, CUBE_VERTICES, CUBE_FACES)


class TriangleMesh(_MeshPrimitive):
    """Arbitrary triangle soup (OBJ meshes, instancing). Normals follow Cube's
    +normalize(e1 x e2) convention unless explicit face normals are given."""
    normal_sign = 1.0
    type_name = "mesh"

    def __init__(self, trans_mat, bsdf, vertices, faces, face_normals=None):
        if face_normals is None:
            super().__init__(trans_mat, bsdf, vertices, faces)
            return
        self.id = -1
        self.trans_mat = trans_mat
        self.bsdf = bsdf
        self.vertices, self.faces = apply_transform(vertices, faces, trans_mat)
        self.normal_vectors = np.asarray(face_normals, np.float32)
        self.bounds = BBox(None, None)
        self.bounds.from_vertices(self.vertices)
        self.center = self.bounds.center()


class Sphere:
    """Analytic sphere (reference intersection_taichi.py:164-181; hit :15-36)."""
    type_name = "sphere"

    def __init__(self, center, radius, bsdf):
        self.id = -1
        self.center = np.asarray(center, np.float64)
        self.radius = float(radius)
        self.bsdf = bsdf
        self.bounds = BBox(self.center - radius, self.center + radius)

    @property
    def bounding_box(self):
        return self.bounds.min_coord, self.bounds.max_coord
