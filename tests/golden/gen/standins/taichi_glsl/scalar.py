"""taichi_glsl.scalar stand-in (FIXTURE-GENERATION ONLY)."""
import numpy as np


def isnan(x):
    return bool(np.isnan(x))


def clamp(x, lo=0.0, hi=1.0):
    return np.minimum(np.maximum(x, lo), hi)
