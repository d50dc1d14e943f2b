"""numba stand-in (FIXTURE-GENERATION ONLY): decorators are identity."""


def njit(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    return lambda f: f


def guvectorize(*args, **kwargs):
    return lambda f: f


def vectorize(*args, **kwargs):
    return lambda f: f





class _Config:
    NUMBA_DEFAULT_NUM_THREADS = 1


class _Sig:
    """`float32[:]` in a signature list: indexable placeholder."""

    def __getitem__(self, key):
        return self


config = _Config()
float32 = _Sig()
float64 = _Sig()
