"""BSDF descriptions (reference: core/bsdf.py:18-91; core/bsdf_taichi.py:45-86).

Host-side records only; sampling/evaluation runs in the HIP kernel.  Each BSDF
packs into one material row of the C-ABI: rho.rgb, emit, sided, type, ior,
roughness (include/prt.h, PRT_MAT_*).

  lambert  -> BSDFLambertian  (rho, emitting_light=0, sided=0)   bsdf.py:18-42
  null     -> BSDFLight       (rho scalar, emitting_light=1, sided=1)  bsdf.py:45-65
  metal    -> BSDFMetal       (bsdf_taichi.py:45-59; build-added, config 3)
  dielectric -> BSDFDielectric (bsdf_taichi.py:62-86; build-added, config 3)

The reference factory raises NotImplementedError for any type other than
lambert/null (bsdf.py:76-78); `BSDF(data, strict=True)` keeps that behaviour.
"""
import numpy as np

MAT_LAMBERT = 0
MAT_LIGHT = 1
MAT_METAL = 2
MAT_DIELECTRIC = 3


class BSDFLambertian:
    type_id = MAT_LAMBERT

    def __init__(self, data):
        a = data["albedo"]
        self.rho = np.array([a[0], a[1], a[2]], np.float32) if not np.isscalar(a) else np.full(3, a, np.float32)
        self.emitting_light = 0
        self.sided = 0

    def evaluate(self):
        return self.rho

    def pack(self):
        return [*self.rho, 0.0, 0.0, float(self.type_id), 1.0, 0.0]


class BSDFLight:
    type_id = MAT_LIGHT

    def __init__(self, data):
        self.rho = data["albedo"]
        self.emitting_light = 1
        self.sided = 1

    def evaluate(self):
        r = np.float32(self.rho)
        return np.array([r, r, r], np.float32)

    def pack(self):
        e = self.evaluate()
        return [*e, 1.0, 1.0, float(self.type_id), 1.0, 0.0]


class BSDFMetal:
    type_id = MAT_METAL

    def __init__(self, data):
        a = data.get("albedo", [1.0, 1.0, 1.0])
        self.rho = np.array(a if not np.isscalar(a) else [a, a, a], np.float32)
        self.roughness = min(float(data.get("roughness", 0.0)), 1.0)
        self.emitting_light = 0
        self.sided = 0

    def evaluate(self):
        return self.rho

    def pack(self):
        return [*self.rho, 0.0, 0.0, float(self.type_id), 1.0, self.roughness]


class BSDFDielectric:
    type_id = MAT_DIELECTRIC

    def __init__(self, data):
        self.ior = float(data.get("ior", 1.5))
        self.rho = np.ones(3, np.float32)
        self.emitting_light = 0
        self.sided = 0

    def evaluate(self):
        return self.rho

    def pack(self):
        return [*self.rho, 0.0, 0.0, float(self.type_id), self.ior, 0.0]


_TYPES = {"lambert": BSDFLambertian, "null": BSDFLight, "metal": BSDFMetal, "dielectric": BSDFDielectric}


class BSDF:
    def __init__(self, data, strict=False):
        self._type = data["type"]
        if self._type not in _TYPES or (strict and self._type not in ("lambert", "null")):
            print(f"[WARNING] bsdf of type {self._type} not implemented")
            raise NotImplementedError(self._type)
        self.distribution = _TYPES[self._type](data)
        self.emitting_light = self.distribution.emitting_light
        self.sided = self.distribution.sided

    def get_distribution(self):
        return self.distribution

    def bsdf_info(self):
        return self.emitting_light, self.sided
