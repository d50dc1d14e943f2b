"""CPU stand-in for the parts of Taichi that pyrenderer's hot path touches.

FIXTURE-GENERATION ONLY.  Taichi is not installed in this image and there is
no network, so `tests/golden/gen/make_golden.py` executes the reference's own
Python source (`/root/reference`) with this module standing in for `taichi`.
It is never imported by the product (`pyrenderer_amd/`), by `bench.py`, or by
any test that runs on the GPU box; only the `.npz` vectors it helps produce are
committed under `tests/golden/`.

Semantics mirrored (Taichi default_fp = f32):
  * `@ti.func` / `@ti.kernel` / `@ti.data_oriented` / `ti.static` are identity;
  * `ti.Vector` values are float32 numpy arrays with `.dot/.cross/.norm/...`;
    arithmetic stays in f32 because numpy 2 treats Python scalars as weak;
  * fields are dense numpy arrays (allocated at `place()` time if unsized);
  * `ti.random()` draws float32 in [0, 1) from a module-level numpy Generator
    that the generator script seeds (`seed_random`).
"""
import numpy as np

f32 = np.float32
f64 = np.float64
i32 = np.int32
i8 = np.int8
u32 = np.uint32
uint32 = np.uint32
int32 = np.int32
i = "i"
ij = "ij"
gpu = "gpu"
cpu = "cpu"

_rng = np.random.default_rng(0)


def seed_random(seed):
    global _rng
    _rng = np.random.default_rng(seed)


_script = None
_script_pos = 0


def script_random(values):
    """Replay a fixed stream of draws (None restores the seeded generator)."""
    global _script, _script_pos
    _script = None if values is None else np.asarray(values, dtype=np.float32)
    _script_pos = 0


def script_consumed():
    return _script_pos


def random(dtype=None):
    global _script_pos
    if _script is not None:
        if _script_pos >= _script.shape[0]:
            raise IndexError("scripted random stream exhausted")
        r = _script[_script_pos]
        _script_pos += 1
        return np.float32(r)
    return np.float32(_rng.random(dtype=np.float32))


def init(*args, **kwargs):
    return None


def func(fn):
    return fn


def kernel(fn):
    return fn


def data_oriented(cls):
    return cls


def static(x):
    return x


def template():
    return None


def sqrt(x):
    return np.sqrt(x)


def abs(x):  # noqa: A001 - mirrors ti.abs
    return np.abs(x)


def cos(x):
    # correctly rounded f32 cosine: the stand-in's choice (Taichi's own cos is
    # backend-dependent); the oracle's "libm" trig mode uses the same rounding.
    return np.float32(np.cos(np.float64(x)))


def sin(x):
    return np.float32(np.sin(np.float64(x)))


def acos(x):
    return np.arccos(x)


def max(a, b):  # noqa: A001
    return np.maximum(a, b)


def min(a, b):  # noqa: A001
    return np.minimum(a, b)


def cast(x, dtype):
    return dtype(x)


class Vec(np.ndarray):
    """float32 small vector with Taichi's Matrix helpers."""

    def __new__(cls, data, dtype=np.float32):
        return np.asarray(data, dtype=dtype).view(cls)

    def __array_finalize__(self, obj):
        pass

    def dot(self, other):
        a = np.asarray(self)
        b = np.asarray(other)
        prod = a * b
        acc = prod[0]
        for k in range(1, prod.shape[0]):
            acc = acc + prod[k]
        return acc

    def cross(self, other):
        a = np.asarray(self)
        b = np.asarray(other)
        return Vec([a[1] * b[2] - a[2] * b[1],
                    a[2] * b[0] - a[0] * b[2],
                    a[0] * b[1] - a[1] * b[0]], dtype=a.dtype)

    def norm_sqr(self):
        return self.dot(self)

    def norm(self):
        return np.sqrt(self.dot(self))

    def normalized(self):
        return self / self.norm()

    def sum(self, *args, **kwargs):
        a = np.asarray(self)
        acc = a[0]
        for k in range(1, a.shape[0]):
            acc = acc + a[k]
        return acc

    @property
    def x(self):
        return self[0]

    @property
    def y(self):
        return self[1]

    @property
    def z(self):
        return self[2]

    def __getitem__(self, key):
        r = np.ndarray.__getitem__(self, key)
        if isinstance(r, np.ndarray) and r.ndim == 0:
            return r[()]
        if isinstance(r, np.ndarray) and not isinstance(key, (int, np.integer)):
            return r.view(Vec)
        return r


class _Field:
    def __init__(self, dtype, n=None, shape=None):
        self.dtype = dtype
        self.n = n
        self.data = None
        if shape is not None:
            self._alloc(shape)

    def _alloc(self, shape):
        if isinstance(shape, int):
            shape = (shape,)
        full = tuple(shape) + ((self.n,) if self.n else ())
        self.data = np.zeros(full, dtype=self.dtype)

    def _key(self, key):
        if isinstance(key, tuple):
            return tuple(int(k) for k in key)
        return int(key)

    def __getitem__(self, key):
        v = self.data[self._key(key)]
        if self.n:
            return Vec(v, dtype=self.dtype)
        return v

    def __setitem__(self, key, value):
        self.data[self._key(key)] = np.asarray(value, dtype=self.dtype)

    def from_numpy(self, arr):
        self.data = np.asarray(arr, dtype=self.dtype).copy()

    def to_numpy(self):
        return self.data.copy()


def field(dtype=np.float32, shape=None):
    return _Field(dtype, None, shape)


class Vector:
    """`ti.Vector([...])` constructs a value; `ti.Vector.field` a field."""

    def __new__(cls, data, dt=None):
        return Vec(data, dtype=dt or np.float32)

    @staticmethod
    def field(n=3, dtype=np.float32, shape=None):
        return _Field(dtype, n, shape)


Matrix = Vector


class _Dense:
    def __init__(self, shape):
        self.shape = shape

    def place(self, *fields):
        for fl in fields:
            fl._alloc(self.shape)


class _Root:
    def dense(self, axes, shape):
        return _Dense(shape)


root = _Root()
