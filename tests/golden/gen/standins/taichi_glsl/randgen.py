"""taichi_glsl.randgen stand-in (FIXTURE-GENERATION ONLY). randInt is inclusive."""
import numpy as np
import taichi as ti


def rand():
    return ti.random()


def randInt(a, b):
    k = int(np.floor(np.float32(rand()) * np.float32(b - a + 1)))
    return a + min(k, b - a)
