"""Tungsten scene JSON loader (reference: io_utils/read_tungsten.py:9-46).

Reads camera (position/look_at/up, resolution, fov), BSDFs and primitives.
Supported primitive types: quad, cube (reference) plus, as build-added
extensions, `sphere` (center/radius in "transform") and `mesh` (OBJ file via
"file").  Unknown types are skipped with the reference's warning.  The JSON
`emission`, `integrator` and `renderer` blocks are ignored, as in the
reference: the directly-hit light colour is core/tracing.py:120's constant and
NEE radiance is BSDFLight.evaluate().
"""
import json
import os

import numpy as np

from ..core.bsdf import BSDF
from ..core.camera import Camera
from ..core.scene import Scene
from ..mathematics.affine_transformation import make_transformation_matrix
from ..mathematics.shapes import Cube, Quad, Sphere, TriangleMesh

PRIM_TYPES = {"quad": Quad, "cube": Cube}


def load_obj(path):
    """Minimal OBJ reader: `v x y z` and `f a b c` / `f a//n ...` (1-based)."""
    verts, faces = [], []
    with open(path) as fh:
        for line in fh:
            parts = line.split()
            if not parts:
                continue
            if parts[0] == "v":
                verts.append([float(x) for x in parts[1:4]])
            elif parts[0] == "f":
                idx = [int(p.split("/")[0]) for p in parts[1:]]
                idx = [i - 1 if i > 0 else len(verts) + i for i in idx]
                for k in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[k], idx[k + 1]])
    return np.asarray(verts, np.float64), np.asarray(faces, np.int64)


def process_primitives(data, base_dir=".", strict_bsdf=False):
    a_scene = Scene()
    cam = data["camera"]
    a_camera = Camera(cam["transform"]["position"], cam["transform"]["look_at"], cam["transform"]["up"],
                      cam["resolution"], fov=cam["fov"])
    name2bsdf = {}
    for info_bsdf in data["bsdfs"]:
        name2bsdf[info_bsdf["name"]] = BSDF(info_bsdf, strict=strict_bsdf).get_distribution()
    for info in data["primitives"]:
        ptype = info["type"]
        if ptype in PRIM_TYPES:
            trans_mat = make_transformation_matrix(info["transform"])
            prim = PRIM_TYPES[ptype](trans_mat, name2bsdf[info["bsdf"]])
        elif ptype == "sphere":
            tr = info.get("transform", {})
            prim = Sphere(tr.get("position", [0, 0, 0]), info.get("radius", tr.get("scale", 1.0)),
                          name2bsdf[info["bsdf"]])
        elif ptype == "mesh" and "file" in info:
            v, f = load_obj(os.path.join(base_dir, info["file"]))
            prim = TriangleMesh(make_transformation_matrix(info.get("transform", {})), name2bsdf[info["bsdf"]], v, f)
        else:
            print(f"[WARNING] {ptype} not implemented")
            continue
        a_scene.add_primitive(prim)
    return a_scene, a_camera


def read_file(filename, strict_bsdf=False):
    with open(filename) as json_file:
        data = json.load(json_file)
    return process_primitives(data, os.path.dirname(os.path.abspath(filename)), strict_bsdf)
