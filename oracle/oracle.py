"""ctypes front-end of the CPU oracle (oracle/prt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package `pyrenderer_amd`.
It is the checker the HIP path is compared against, and the "port" CPU
baseline timed beside the GPU number.

Parity status: pinned.  The restatement is checked against vectors produced by
the reference's own code (tests/golden/*.npz, generator committed under
tests/golden/gen/): the 9 recorded bounces of test.py:38-57, ~3k World.hit_all
queries, unit known-answer vectors, PathTracer.trace replayed on scripted random
streams, and a statistical image of main_taichi.py's render().
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PRT_ORACLE_LIB: another build of the same source (tools/sanitize: AddressSanitizer + UBSan)
_LIB_PATH = os.environ.get("PRT_ORACLE_LIB") or os.path.join(_HERE, "_build", "libprt_oracle.so")

BACKEND_REF = 0     # reference structure: median-split BVH over primitives + per-primitive loop
BACKEND_BRUTE = 1   # all triangles, closest (t, index)
BACKEND_BVH = 2     # stack traversal of an external BVH2 (prt_bvh_export arrays); boxes only prune

_f = ctypes.c_float
_i = ctypes.c_int
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_vp = ctypes.c_void_p


def build():
    """Compile oracle/_build/libprt_oracle.so with oracle/Makefile."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.or_scene_create.restype = _vp
        L.or_scene_create.argtypes = [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _i64, _vp, _i32, _vp, _vp,
                                      _i32, _vp]
        L.or_scene_destroy.argtypes = [_vp]
        L.or_set_trig_mode.argtypes = [_i]
        L.or_scene_set_bvh.argtypes = [_vp, _vp, _i64, _vp, _i64]
        L.or_ref_bvh.argtypes = [_vp] + [_vp] * 6
        L.or_mt.argtypes = [_vp] * 5 + [_f, _f, _vp]
        L.or_aabb.argtypes = [_vp] * 4 + [_f, _f]
        L.or_disk.argtypes = [_vp, _vp]
        L.or_hemi.argtypes = [_vp, _vp]
        L.or_frame.argtypes = [_vp, _vp]
        L.or_rotate.argtypes = [_vp, _vp, _vp]
        L.or_gen_ray.argtypes = [_vp, _f, _f, _vp, _vp]
        L.or_sphere.argtypes = [_vp, _f, _vp, _vp, _f, _f, _vp]
        L.or_reflect.argtypes = [_vp, _vp, _vp]
        L.or_refract.argtypes = [_vp, _vp, _f, _vp]
        L.or_schlick.argtypes = [_f, _f]
        L.or_schlick.restype = _f
        L.or_rng_key.argtypes = [_u64, _u32, _u32]
        L.or_rng_key.restype = _u32
        L.or_rng_draws.argtypes = [_u32, _i, _vp]
        L.or_sample_light_scripted.argtypes = [_vp, _vp, _vp, _vp, _vp]
        L.or_closest_batch.argtypes = [_vp, _i, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        L.or_trace_scripted.argtypes = [_vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _vp]
        L.or_render_tiles.argtypes = [_vp, _i, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _u64, _i, _vp, _vp]
        L.or_set_nee_mode.argtypes = [_i]
        L.or_mis_power.argtypes = [_f, _f]
        L.or_mis_power.restype = _f
        L.or_area_light_pdf.argtypes = [_f, _vp, _vp]
        L.or_area_light_pdf.restype = _f
        L.or_brdf_pdf.argtypes = [_vp, _vp]
        L.or_brdf_pdf.restype = _f
        L.or_dot_or_zero.argtypes = [_vp, _vp]
        L.or_dot_or_zero.restype = _f
        L.or_direct_mis_scripted.argtypes = [_vp, _vp, _vp, _vp, _vp, _i, _vp]
        L.or_hit_all_batch.argtypes = [_vp, _i, _i64, _vp, _vp, _vp, _vp, _u64, _vp]
        L.or_trace_rays.argtypes = [_vp, _i, _i64, _vp, _vp, _i, _u64, _i, _vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_vp)


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a if shape is None else a.reshape(shape)


class OracleScene:
    """Oracle view of a flattened scene (same arrays the C-ABI takes).

    tri_v (n,9) f32 world vertices v0 v1 v2; tri_n (n,3) face normals;
    tri_mat (n,) material ids; tri_prim (n,) primitive ids (contiguous, in
    insertion order — needed by the reference-structure backend);
    prim_lo / prim_hi (n_prim,3) f32 primitive bounds; mat (n_mat,8) rows
    rho.rgb, emit, sided, type, ior, roughness; light_tri / light_off per-light
    face lists; direct_rgb the directly-hit light colour (core/tracing.py:120).
    """

    def __init__(self, tri_v, tri_n, tri_mat, tri_prim, prim_lo, prim_hi, mat, light_tri, light_off, direct_rgb,
                 sph=None, sph_mat=None):
        sph = np.zeros((0, 4), np.float32) if sph is None else sph
        sph_mat = np.zeros(0, np.int32) if sph_mat is None else sph_mat
        self._keep = [_f32(tri_v, (-1, 9)), _f32(tri_n, (-1, 3)), np.ascontiguousarray(tri_mat, np.int32),
                      np.ascontiguousarray(tri_prim, np.int32), _f32(prim_lo, (-1, 3)), _f32(prim_hi, (-1, 3)),
                      _f32(mat, (-1, 8)), np.ascontiguousarray(light_tri, np.int32),
                      np.ascontiguousarray(light_off, np.int32), _f32(direct_rgb, (3,)),
                      _f32(sph, (-1, 4)), np.ascontiguousarray(sph_mat, np.int32)]
        k = self._keep
        self.n_tri = k[0].shape[0]
        self.n_prim = k[4].shape[0]
        self.h = lib().or_scene_create(_p(k[0]), _p(k[1]), _p(k[2]), _p(k[3]), self.n_tri, _p(k[4]), _p(k[5]),
                                       self.n_prim, _p(k[10]), _p(k[11]), k[10].shape[0], _p(k[6]), k[6].shape[0],
                                       _p(k[7]), _p(k[8]), k[8].shape[0] - 1, _p(k[9]))

    @classmethod
    def from_flat(cls, flat):
        """Build from a pyrenderer_amd FlatScene-like object or dict."""
        g = flat if isinstance(flat, dict) else flat.__dict__
        return cls(g["tri_v"], g["tri_n"], g["tri_mat"], g["tri_prim"], g["prim_lo"], g["prim_hi"], g["mat"],
                   g["light_tri"], g["light_off"], g["direct_rgb"], g.get("sph"), g.get("sph_mat"))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_scene_destroy(self.h)
            self.h = None

    def set_bvh(self, nodes, order):
        """Attach BVH2 arrays (from pyrenderer_amd's prt_bvh_export) for BACKEND_BVH."""
        nodes = _f32(nodes, (-1, 16))
        order = np.ascontiguousarray(order, np.int32)
        self._keep += [nodes, order]
        lib().or_scene_set_bvh(self.h, _p(nodes), nodes.shape[0], _p(order), order.shape[0])

    def ref_bvh(self):
        n = 2 * self.n_prim
        obj, left, right, nxt = (np.zeros(n, np.int32) for _ in range(4))
        mn = np.zeros((n, 3), np.float32)
        mx = np.zeros((n, 3), np.float32)
        cnt = lib().or_ref_bvh(self.h, _p(obj), _p(left), _p(right), _p(nxt), _p(mn), _p(mx))
        return dict(obj=obj[:cnt], left=left[:cnt], right=right[:cnt], next=nxt[:cnt], min=mn[:cnt], max=mx[:cnt])

    def closest(self, ro, rd, tmin, tmax, backend=BACKEND_BRUTE):
        ro = _f32(ro, (-1, 3))
        rd = _f32(rd, (-1, 3))
        n = ro.shape[0]
        t0 = _f32(np.broadcast_to(tmin, (n,)))
        t1 = _f32(np.broadcast_to(tmax, (n,)))
        hit = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        tri = np.zeros(n, np.int64)
        nrm = np.zeros((n, 3), np.float32)
        lib().or_closest_batch(self.h, backend, n, _p(ro), _p(rd), _p(t0), _p(t1), _p(hit), _p(t), _p(tri), _p(nrm))
        return hit, t, tri, nrm

    def hit_all(self, ro, rd, tmin, tmax, seed=0, backend=BACKEND_BRUTE):
        """World.hit_all's 8-tuple per ray as libprt's prt_hit_all: (n, 16) f32 rows = hit, t, p,
        normal, emit, attenuation, scattered direction, pdf (scatter keyed (seed, i, 0))."""
        ro = _f32(ro, (-1, 3))
        rd = _f32(rd, (-1, 3))
        n = ro.shape[0]
        t0 = _f32(np.broadcast_to(tmin, (n,)))
        t1 = _f32(np.broadcast_to(tmax, (n,)))
        out = np.zeros((n, 16), np.float32)
        lib().or_hit_all_batch(self.h, backend, n, _p(ro), _p(rd), _p(t0), _p(t1), int(seed), _p(out))
        return out

    def trace_rays(self, ro, rd, depth, seed=0, backend=BACKEND_BRUTE, nthreads=0):
        """PathTracer.trace per caller ray as libprt's prt_trace_rays: (n, 3) radiance."""
        ro = _f32(ro, (-1, 3))
        rd = _f32(rd, (-1, 3))
        out = np.zeros((ro.shape[0], 3), np.float32)
        lib().or_trace_rays(self.h, backend, ro.shape[0], _p(ro), _p(rd), depth, int(seed), nthreads, _p(out))
        return out

    def sample_light_scripted(self, draws):
        d = np.zeros(16, np.float32)
        d[:len(draws)] = draws
        p2 = np.zeros(3, np.float32)
        n2 = np.zeros(3, np.float32)
        e = np.zeros(3, np.float32)
        lib().or_sample_light_scripted(self.h, _p(d), _p(p2), _p(n2), _p(e))
        return p2, n2, e

    def direct_mis_scripted(self, p, n, rho, stream):
        """sample_direct_lighting2 on a scripted stream: (direct radiance, draws consumed)."""
        stream = _f32(stream)
        out = np.zeros(3, np.float32)
        used = lib().or_direct_mis_scripted(self.h, _p(_f32(p)), _p(_f32(n)), _p(_f32(rho)), _p(stream),
                                            stream.shape[0], _p(out))
        return out, used

    def trace_scripted(self, cam, W, H, x, y, depth, stream):
        stream = _f32(stream)
        out = np.zeros(3, np.float32)
        cam = _f32(cam)
        used = lib().or_trace_scripted(self.h, _p(cam), W, H, int(x), int(y), depth, _p(stream), stream.shape[0],
                                       _p(out))
        return out, used

    def render_tiles(self, cam, W, H, tw, th, tile_ids, spp, depth, seed=0, backend=BACKEND_BRUTE, nthreads=0,
                     counters=False):
        """Sequential per-pixel sums over spp samples, slot order of prt_render_tiles."""
        cam = _f32(cam)
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        out = np.zeros((tile_ids.shape[0] * tw * th, 3), np.float32)
        cnt = np.zeros(4, np.uint64)
        lib().or_render_tiles(self.h, backend, _p(cam), W, H, tw, th, _p(tile_ids), tile_ids.shape[0], spp, depth,
                              seed, nthreads, _p(out), _p(cnt) if counters else None)
        return (out, cnt) if counters else out

    def render(self, cam, W, H, spp, depth, seed=0, backend=BACKEND_BRUTE, nthreads=0, tile=64):
        """Full frame, returned as per-pixel SUMS in the reference layout (W, H, 3), [x][y]."""
        tx = (W + tile - 1) // tile
        ty = (H + tile - 1) // tile
        ids = np.arange(tx * ty, dtype=np.int32)
        slots = self.render_tiles(cam, W, H, tile, tile, ids, spp, depth, seed, backend, nthreads)
        return unpack_tiles(slots, W, H, tile, tile, ids)


def unpack_tiles(slots, W, H, tw, th, tile_ids):
    """Slot-ordered (n_tiles*tw*th, 3) → (W, H, 3) frame indexed [x][y]."""
    tx = (W + tw - 1) // tw
    frame = np.zeros((W, H, 3), np.float32)
    s = slots.reshape(len(tile_ids), th, tw, 3)
    for k, tid in enumerate(tile_ids):
        x0 = (tid % tx) * tw
        y0 = (tid // tx) * th
        w = min(tw, W - x0)
        h = min(th, H - y0)
        frame[x0:x0 + w, y0:y0 + h] = s[k, :h, :w].transpose(1, 0, 2)
    return frame


def set_nee_mode(mis):
    """False = sample_direct_lighting (the path the reference's trace runs); True = the
    MIS variant sample_direct_lighting2 (core/tracing.py:57-90) in its place."""
    lib().or_set_nee_mode(1 if mis else 0)


def mis_power(pf, pg):
    return lib().or_mis_power(float(pf), float(pg))


def area_light_pdf(t, d, n2):
    return lib().or_area_light_pdf(float(t), _p(_f32(d)), _p(_f32(n2)))


def brdf_pdf(n, d):
    return lib().or_brdf_pdf(_p(_f32(n)), _p(_f32(d)))


def dot_or_zero(n, d):
    return lib().or_dot_or_zero(_p(_f32(n)), _p(_f32(d)))


def set_trig_mode(mode):
    """0 = spec polynomials (shared with the HIP kernel); 1 = correctly rounded
    libm trig on the reference's literal theta (reference replays only)."""
    lib().or_set_trig_mode(int(mode))


# ------------------------------------------------------------- unit kernels
def mt(v0, v1, v2, ro, rd, t0, t1):
    t = np.zeros(1, np.float32)
    h = lib().or_mt(_p(_f32(v0)), _p(_f32(v1)), _p(_f32(v2)), _p(_f32(ro)), _p(_f32(rd)), float(t0), float(t1), _p(t))
    return h, t[0]


def aabb(lo, hi, ro, rd, t0, t1):
    return lib().or_aabb(_p(_f32(lo)), _p(_f32(hi)), _p(_f32(ro)), _p(_f32(rd)), float(t0), float(t1))


def disk(u):
    o = np.zeros(2, np.float32)
    lib().or_disk(_p(_f32(u)), _p(o))
    return o


def hemi(u):
    o = np.zeros(3, np.float32)
    lib().or_hemi(_p(_f32(u)), _p(o))
    return o


def frame(n):
    o = np.zeros(9, np.float32)
    lib().or_frame(_p(_f32(n)), _p(o))
    return o.reshape(3, 3)


def rotate(rows, v):
    o = np.zeros(3, np.float32)
    lib().or_rotate(_p(_f32(rows)), _p(_f32(v)), _p(o))
    return o


def gen_ray(cam, u, v):
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    lib().or_gen_ray(_p(_f32(cam)), float(u), float(v), _p(o), _p(d))
    return o, d


def sphere(c, r, ro, rd, t0, t1):
    root = np.zeros(1, np.float32)
    h = lib().or_sphere(_p(_f32(c)), float(r), _p(_f32(ro)), _p(_f32(rd)), float(t0), float(t1), _p(root))
    return h, root[0]


def reflect(v, n):
    o = np.zeros(3, np.float32)
    lib().or_reflect(_p(_f32(v)), _p(_f32(n)), _p(o))
    return o


def refract(v, n, eta):
    o = np.zeros(3, np.float32)
    lib().or_refract(_p(_f32(v)), _p(_f32(n)), float(eta), _p(o))
    return o


def schlick(c, idx):
    return lib().or_schlick(float(c), float(idx))


def rng_key(seed, pixel, sample):
    return lib().or_rng_key(seed, pixel, sample)


def rng_draws(key, n):
    o = np.zeros(n, np.float32)
    lib().or_rng_draws(key, n, _p(o))
    return o
