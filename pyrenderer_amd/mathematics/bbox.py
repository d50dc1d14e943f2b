"""Axis-aligned bounds (reference: mathematics/bbox.py:27-73, host side only)."""
import numpy as np

from .constants import EPS, MAX_F


class BBox:
    def __init__(self, min_coord=None, max_coord=None):
        if min_coord is None:
            self.min_coord = np.array([MAX_F, MAX_F, MAX_F])
            self.max_coord = self.min_coord * -1
        else:
            self.min_coord = np.asarray(min_coord)
            self.max_coord = np.asarray(max_coord)
        self.empty = False

    def from_vertices(self, vertices):
        self.min_coord = np.min(vertices, axis=0)
        self.max_coord = np.max(vertices, axis=0)
        self.update_empty()

    def update_empty(self):
        self.empty = bool(np.any(np.abs(self.min_coord - self.max_coord) <= EPS))

    def center(self):
        return (self.min_coord + self.max_coord) / 2.0

    def is_empty(self):
        return self.empty

    def enclose(self, other):
        self.min_coord = np.minimum(self.min_coord, other.min_coord)
        self.max_coord = np.maximum(self.max_coord, other.max_coord)
        self.update_empty()

    def surface_area(self):
        e = self.max_coord - self.min_coord
        return 2.0 * (e[0] * e[2] + e[0] * e[1] + e[1] * e[2])

    def __str__(self):
        return f"bbox: max={self.max_coord} min={self.min_coord}"
