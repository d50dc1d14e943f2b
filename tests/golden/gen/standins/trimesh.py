"""trimesh stand-in (FIXTURE-GENERATION ONLY): Trimesh(vertices, faces) + apply_transform.

apply_transform = (M @ [v, 1]^T)^T in float64; if det(M[:3,:3]) < 0 the face
winding is reversed (trimesh behaviour; never triggered by the Cornell scene).
"""
import numpy as np


class Trimesh:
    def __init__(self, vertices=None, faces=None, process=False):
        self.vertices = np.asarray(vertices, dtype=np.float64)
        self.faces = np.asarray(faces)

    def apply_transform(self, matrix):
        m = np.asarray(matrix, dtype=np.float64)
        homo = np.hstack([self.vertices, np.ones((self.vertices.shape[0], 1))])
        self.vertices = np.dot(m, homo.T).T[:, :3]
        if np.linalg.det(m[:3, :3]) < 0:
            self.faces = np.ascontiguousarray(self.faces[:, ::-1])
        return self

    def show(self):
        pass
