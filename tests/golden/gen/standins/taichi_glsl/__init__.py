"""CPU stand-in for taichi_glsl (FIXTURE-GENERATION ONLY; see ../taichi/__init__.py).

`randInt(a, b)` is taken as INCLUSIVE of b (SURVEY.md §7 hard parts: the
taichi_glsl source is not available offline, so this is an assumption that the
build documents as "parity unpinned" for light-face selection).
"""
from .vector import vec2, vec3, vec4, normalize, dot, cross, sqrLength, reflect, length  # noqa: F401
from .scalar import isnan, clamp  # noqa: F401
from .randgen import rand, randInt  # noqa: F401
import taichi as _ti

mat = _ti.Vector
