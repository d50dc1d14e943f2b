"""pyrr.matrix44 stand-in: create_look_at in pyrr's row-vector layout."""
import numpy as np


def _normalize(v):
    return v / np.sqrt(np.sum(v * v))


def create_look_at(eye, target, up, dtype=None):
    eye = np.asarray(eye)
    target = np.asarray(target)
    up = np.asarray(up)
    forward = _normalize(target - eye)
    side = _normalize(np.cross(forward, up))
    up = _normalize(np.cross(side, forward))
    return np.array(((side[0], up[0], -forward[0], 0.),
                     (side[1], up[1], -forward[1], 0.),
                     (side[2], up[2], -forward[2], 0.),
                     (-np.dot(side, eye), -np.dot(up, eye), np.dot(forward, eye), 1.0)), dtype=dtype)


def create_from_eulers(eulers, dtype=None):
    raise NotImplementedError
