"""taichi_glsl.vector stand-in (FIXTURE-GENERATION ONLY)."""
import numpy as np
import taichi as ti


def vec2(*a):
    return ti.Vec(a if len(a) > 1 else [a[0], a[0]])


def vec3(*a):
    return ti.Vec(a if len(a) > 1 else [a[0]] * 3)


def vec4(*a):
    return ti.Vec(a if len(a) > 1 else [a[0]] * 4)


def dot(a, b):
    return ti.Vec(a).dot(b)


def cross(a, b):
    return ti.Vec(a).cross(b)


def sqrLength(v):
    return ti.Vec(v).dot(v)


def length(v):
    return np.sqrt(sqrLength(v))


def normalize(v):
    v = ti.Vec(v)
    return v / length(v)


def reflect(i, n):
    return i - 2.0 * dot(n, i) * n
