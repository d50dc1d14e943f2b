"""NumPy restatement of the render path — the "main.py NumPy path" CPU baseline.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg, never
by the product package `pyrenderer_amd`.

The reference's main.py drives a NumPy/numba per-pixel tracer with joblib workers
(main.py:40-59, n_jobs=4).  SURVEY.md §8(d) asks for the build's NumPy counterpart,
vectorised over ray batches and run with one process per core, timed beside the GPU
number.  This module is that counterpart: PathTracer.trace (core/tracing.py:116-155)
and the render() sample body (main_taichi.py:89-95) as array code over every path of
a batch at once, with the same f32 arithmetic contract as oracle/prt_oracle.c (one
rounding per operation, the reference's expression order, the PCG streams keyed by
(seed, pixel, sample), the minimax sin/cos of the concentric map), so its sums are
bit-identical to the C oracle and therefore to the HIP kernel
(tests/test_numpy_path.py).

Scope: triangle scenes (<= 4096 triangles) with Lambertian and light BSDFs (BASELINE configs 1,
2 and 5),
pinhole cameras; closest hit by brute force over all triangles (closest (t, index),
which is what every backend of the oracle returns).  Specular BSDFs, spheres and thin
lenses raise NotImplementedError.

Per-function references (the C oracle function each block restates):
  _rng_next / _rng_int        prt_oracle.c:98-114  (taichi ti.random / randInt)
  _mt                         prt_oracle.c:129-150 (intersection_taichi.py:69-91)
  _cosine_hemisphere          prt_oracle.c:177-204 (samplers.py:9-32)
  _frame_rotate               prt_oracle.c:207-224 (mat4_taichi.py:9-60)
  _gen_ray                    prt_oracle.c:228-248 (camera_taichi.py:47-74)
  _sample_light               prt_oracle.c:684-701 (intersection_taichi.py:194-207, shapes.py:62-71)
  render_tiles / _trace       prt_oracle.c:704-801, 876-908 (tracing.py:92-155, main_taichi.py:80-99)
"""
import numpy as np

F = np.float32
U = np.uint32
K_INV_PI = F(0.31830988618379067154)
K_PI_OVER_4 = F(0.78539816339744830961)
K_TMIN = F(0.00001)
K_TMAX = F(99999.9)
MAX_F = F(3.402823466e+38)
MAX_TRIANGLES = 4096   # brute force: Cornell-class scenes only
_S = (F(-1.9515295891e-4), F(8.3321608736e-3), F(1.6666654611e-1))
_C = (F(2.443315711809948e-5), F(1.388731625493765e-3), F(4.166664568298827e-2))


# ------------------------------------------------------------------ vectors (N, 3) f32
def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def _cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def _normalize(a):
    return a / np.sqrt(_dot(a, a))[..., None]


# ------------------------------------------------------------------------------ RNG
def _pcg_permute(s):
    w = ((s >> ((s >> U(28)) + U(4))) ^ s) * U(277803737)
    return (w >> U(22)) ^ w


def _pcg_hash(v):
    return _pcg_permute(v * U(747796405) + U(2891336453))


def rng_key(seed, pixel, sample):
    h = _pcg_hash(np.full_like(pixel, U(seed & 0xFFFFFFFF)))
    h = _pcg_hash(h ^ U((seed >> 32) & 0xFFFFFFFF) ^ pixel)
    return _pcg_hash(h + U(sample))


def _rng_next(st, idx):
    """Advance the streams of paths `idx` (in place) and return one uniform each."""
    s = st[idx] * U(747796405) + U(2891336453)
    st[idx] = s
    return (_pcg_permute(s) >> U(8)).astype(F) * F(2.0 ** -24)


def _rng_int(st, idx, a, b):
    u = _rng_next(st, idx)
    k = np.floor(u * F(b - a + 1)).astype(np.int64)
    return a + np.minimum(k, b - a)


# ------------------------------------------------------------------------ kernels
def _poly_sin(x):
    z = x * x
    return (((_S[0] * z + _S[1]) * z - _S[2]) * z) * x + x


def _poly_cos(x):
    z = x * x
    return ((((_C[0] * z - _C[1]) * z + _C[2]) * z) * z - F(0.5) * z) + F(1.0)


def _cosine_hemisphere(u0, u1):
    ox = F(2.0) * u0 - F(1.0)
    oy = F(2.0) * u1 - F(1.0)
    # both branches are evaluated for every lane; the unused one may divide by 0
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        big_x = np.abs(ox) > np.abs(oy)
        th_x = K_PI_OVER_4 * (oy / ox)
        a_y = K_PI_OVER_4 * (ox / oy)
        c = np.where(big_x, _poly_cos(th_x), _poly_sin(a_y))
        s = np.where(big_x, _poly_sin(th_x), _poly_cos(a_y))
    r = np.where(big_x, ox, oy)
    zero = (ox == F(0.0)) & (oy == F(0.0))
    dx = np.where(zero, F(0.0), r * c)
    dy = np.where(zero, F(0.0), r * s)
    m = (F(1.0) - dx * dx) - dy * dy
    return np.stack([dx, dy, np.sqrt(np.where(m > F(0.0), m, F(0.0)))], axis=-1)


def _frame_rotate(n, l):
    """rotate_vector(rotate_z_to(n), l): rows (x, z, v) of the normal frame."""
    v = _normalize(n)
    up = np.zeros_like(v)
    up[:, 1] = F(1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        x = _normalize(_cross(v, up))
        z = _normalize(_cross(x, v))
    pos = (v[:, 1] == F(1.0))[:, None]
    negy = (v[:, 1] == F(-1.0))[:, None]
    ex = np.array([1, 0, 0], F)
    ez = np.array([0, 0, 1], F)
    r1 = np.where(pos | negy, ex, x)
    r2 = np.where(pos | negy, ez, z)
    r3 = np.where(pos, np.array([0, 1, 0], F), np.where(negy, np.array([0, -1, 0], F), v))
    o = (r1 * l[:, 0:1] + r2 * l[:, 1:2]) + r3 * l[:, 2:3]
    return _normalize(o)


def _gen_ray(cam, u, v):
    c = [cam[4 * i:4 * i + 4] for i in range(4)]
    sd = cam[16:20]
    rdir = [((u - F(0.5)) * sd[0]) / F(0.5), ((v - F(0.5)) * sd[1]) / F(0.5), np.full_like(u, -sd[2]),
            np.full_like(u, F(1.0))]
    rorg = [F(0.0), F(0.0), F(0.0), F(1.0)]
    dw = [((rdir[0] * ci[0] + rdir[1] * ci[1]) + rdir[2] * ci[2]) + rdir[3] * ci[3] for ci in c]
    ow = [((rorg[0] * ci[0] + rorg[1] * ci[1]) + rorg[2] * ci[2]) + rorg[3] * ci[3] for ci in c]
    f = [dw[i] - ow[i] for i in range(4)]
    ln = np.sqrt(((f[0] * f[0] + f[1] * f[1]) + f[2] * f[2]) + f[3] * f[3])
    o = np.broadcast_to(np.array(ow[:3], F), (u.shape[0], 3)).copy()
    return o, np.stack([f[0] / ln, f[1] / ln, f[2] / ln], axis=-1)


class NumpyScene:
    """Flattened triangle scene (pyrenderer_amd.flatten output) in the oracle's layout."""

    def __init__(self, flat):
        g = flat if isinstance(flat, dict) else flat.__dict__
        tv = np.asarray(g["tri_v"], F).reshape(-1, 9)
        self.v0 = tv[:, 0:3].copy()
        self.e1 = tv[:, 3:6] - tv[:, 0:3]
        self.e2 = tv[:, 6:9] - tv[:, 0:3]
        self.vtx = tv
        self.nrm = np.asarray(g["tri_n"], F).reshape(-1, 3)
        self.mat_id = np.asarray(g["tri_mat"], np.int64)
        self.mat = np.asarray(g["mat"], F).reshape(-1, 8)
        self.light_tri = np.asarray(g["light_tri"], np.int64)
        self.light_off = np.asarray(g["light_off"], np.int64)
        self.n_light = self.light_off.shape[0] - 1
        self.direct = np.asarray(g["direct_rgb"], F).reshape(3)
        sph = g.get("sph")
        if sph is not None and np.asarray(sph).reshape(-1, 4).shape[0]:
            raise NotImplementedError("numpy path: spheres (config 3) are out of its scope")
        if self.v0.shape[0] > MAX_TRIANGLES:
            raise NotImplementedError(f"numpy path: brute-force closest hit over {self.v0.shape[0]} triangles "
                                      f"(> {MAX_TRIANGLES}; config 4) is out of its scope")
        if np.any((self.mat[:, 5] == 2.0) | (self.mat[:, 5] == 3.0)):
            raise NotImplementedError("numpy path: metal / dielectric BSDFs (config 3) are out of its scope")

    # -------------------------------------------------------------- ray queries
    def _mt(self, ro, rd, t0, t1, chunk=8192):
        """Closest (t, index) over all triangles with the strict t0 < t < t1 test
        (sequential shrinking == min t, lowest index among equal t)."""
        n = ro.shape[0]
        hit = np.zeros(n, bool)
        best_t = t1.copy()
        best_i = np.zeros(n, np.int64)
        for a in range(0, n, chunk):
            o = ro[a:a + chunk, None, :]
            d = rd[a:a + chunk, None, :]
            c = _cross(self.e1[None], d)
            det = _dot(c, self.e2[None])
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                f = F(1.0) / det
                s = o - self.v0[None]
                q = _cross(s, self.e2[None])
                t = -f * _dot(q, self.e1[None])
                u = -f * _dot(q, d)
                v = f * _dot(c, s)
                ok = (np.abs(det) > F(0.0)) & (t0[a:a + chunk, None] < t) & (t < t1[a:a + chunk, None])
                ok &= (F(0.0) <= u) & (u <= F(1.0)) & (v >= F(0.0)) & ((F(1.0) - u) - v >= F(0.0))
            tt = np.where(ok, t, np.inf)
            i = np.argmin(tt, axis=1)
            tb = tt[np.arange(tt.shape[0]), i]
            h = np.isfinite(tb)
            hit[a:a + chunk] = h
            best_t[a:a + chunk] = np.where(h, tb, t1[a:a + chunk])
            best_i[a:a + chunk] = i
        return hit, best_t, best_i

    def _sample_light(self, st, idx):
        m = idx.shape[0]
        li = _rng_int(st, idx, 0, self.n_light - 1) if self.n_light > 1 else np.zeros(m, np.int64)
        nf = self.light_off[li + 1] - self.light_off[li]
        # rng_int(0, nf - 1) with a per-path upper bound
        u = _rng_next(st, idx)
        k = np.minimum(np.floor(u * nf.astype(F)).astype(np.int64), nf - 1)
        tri = self.light_tri[self.light_off[li] + k]
        uu = np.sqrt(_rng_next(st, idx))
        vv = _rng_next(st, idx)
        a = uu * (F(1.0) - vv)
        b = uu * vv
        c = (F(1.0) - a) - b
        t = self.vtx[tri]
        p2 = (t[:, 0:3] * a[:, None] + t[:, 3:6] * b[:, None]) + t[:, 6:9] * c[:, None]
        return p2, self.nrm[tri], self.mat[self.mat_id[tri], 0:3]

    # ------------------------------------------------------------------ render
    def render_pixels(self, cam, W, H, xs, ys, sample, depth, seed=0):
        """Radiance of `sample` for pixels (xs, ys): PathTracer.trace over the batch."""
        cam = np.asarray(cam, F).reshape(-1)
        if cam[19] > 0.0:
            raise NotImplementedError("numpy path: thin-lens cameras are out of its scope")
        n = xs.shape[0]
        st = rng_key(seed, (ys.astype(U) * U(W) + xs.astype(U)), sample)
        allp = np.arange(n)
        r0 = _rng_next(st, allp)
        u = (xs.astype(F) + r0) / F(W - 1)
        r1 = _rng_next(st, allp)
        v = (ys.astype(F) + r1) / F(H - 1)
        ro, rd = _gen_ray(cam, u, v)
        L = np.zeros((n, 3), F)
        beta = np.ones((n, 3), F)
        act = allp
        for b in range(depth):
            if act.size == 0:
                break
            o, d = ro[act], rd[act]
            hit, t, tri = self._mt(o, d, np.full(act.size, K_TMIN), np.full(act.size, K_TMAX))
            act, o, d, t, tri = act[hit], o[hit], d[hit], t[hit], tri[hit]
            m = self.mat[self.mat_id[tri]]
            ng = self.nrm[tri]
            flip = (m[:, 4] == F(0.0)) & (_dot(ng, -d) < F(0.0))
            nn = np.where(flip[:, None], -ng, ng)
            # emitters: tracing.py:129-139, the path ends
            em = m[:, 3] != F(0.0)
            if em.any():
                e_idx, e_n, e_d = act[em], nn[em], d[em]
                d1 = _dot(-e_d, e_n)
                lc = self.direct[None] * beta[e_idx]
                add = lc if b == 0 else lc * d1[:, None]
                pos = d1 > F(0.0)
                L[e_idx[pos]] = L[e_idx[pos]] + add[pos]
            keep = ~em
            act, o, d, t, nn, m = act[keep], o[keep], d[keep], t[keep], nn[keep], m[keep]
            if act.size == 0:
                break
            # BSDFLambertian.scatter + frame (bsdf.py:29-34, shapes.py:105-108)
            u0 = _rng_next(st, act)
            u1 = _rng_next(st, act)
            wi = _frame_rotate(nn, _cosine_hemisphere(u0, u1))
            pdf = np.abs(_dot(nn, wi)) * K_INV_PI
            p = o + d * t[:, None]
            att = m[:, 0:3]
            cw = _dot(nn, wi)
            dz = np.where(cw > F(0.0), cw, F(0.0))
            with np.errstate(divide="ignore", invalid="ignore"):
                nb = ((att * dz[:, None]) / pdf[:, None]) * K_INV_PI
                bad = np.isnan(nb).any(axis=1)
                if bad.any():
                    nb[bad] = ((att[bad] * dz[bad, None]) / F(1e-4)) * K_INV_PI
            beta[act] = beta[act] * nb
            # sample_direct_lighting (tracing.py:92-108)
            p2, n2, e = self._sample_light(st, act)
            w = _normalize(p2 - p)
            w2 = _normalize(p - p2)
            with np.errstate(divide="ignore", invalid="ignore"):
                t_at = (p2[:, 0] - p[:, 0]) / w[:, 0]
            dot1 = _dot(nn, w)
            dot2 = _dot(n2, w2)
            cand = (dot1 > F(0.0)) & (dot2 > F(0.0))
            if cand.any():
                ci = np.nonzero(cand)[0]
                blocked, _, _ = self._mt(p[ci], w[ci], np.full(ci.size, K_TMIN), t_at[ci])
                ci = ci[~blocked]
                dd = p[ci] - p2[ci]
                sl = _dot(dd, dd)
                rad = ((e[ci] * dot1[ci, None]) * dot2[ci, None]) / sl[:, None]
                L[act[ci]] = L[act[ci]] + beta[act[ci]] * rad
            ro[act] = p
            rd[act] = wi
        return L

    def render_tiles(self, cam, W, H, tw, th, tile_ids, spp, depth, seed=0):
        """Per-pixel sums over samples 0..spp-1 in sample order, slot order of prt_render_tiles."""
        tile_ids = np.asarray(tile_ids, np.int64)
        tiles_x = (W + tw - 1) // tw
        loc = np.arange(tw * th)
        xs = ((tile_ids[:, None] % tiles_x) * tw + loc[None] % tw).reshape(-1)
        ys = ((tile_ids[:, None] // tiles_x) * th + loc[None] // tw).reshape(-1)
        inside = (xs < W) & (ys < H)
        out = np.zeros((xs.shape[0], 3), F)
        xi, yi = xs[inside], ys[inside]
        acc = np.zeros((xi.shape[0], 3), F)
        for s in range(spp):
            acc = acc + self.render_pixels(cam, W, H, xi, yi, s, depth, seed)
        out[inside] = acc
        return out


def _tiles_worker(job):
    """One pool task: (flat dict, cam, W, H, tile ids, spp, depth, seed) -> (sums, seconds)."""
    import time
    flat, cam, W, H, ids, spp, depth, seed = job
    sc = NumpyScene(flat)
    t0 = time.perf_counter()
    sums = sc.render_tiles(cam, W, H, 8, 8, ids, spp, depth, seed)
    return sums, time.perf_counter() - t0


def timed_sample(flat, cam, W, H, spp, depth, seed, seconds, procs, rng_seed=2):
    """The NumPy path on a bounded sample of the frame, one process per core (main.py's
    joblib pixel parallelism): random 8x8 tiles sized to about `seconds` of wall time on
    `procs` spawned workers.  Returns (tile ids, per-slot sums, wall seconds)."""
    import multiprocessing as mp
    import time
    g = flat if isinstance(flat, dict) else flat.__dict__
    fd = {k: g[k] for k in ("tri_v", "tri_n", "tri_mat", "mat", "light_tri", "light_off", "direct_rgb", "sph")
          if k in g}
    NumpyScene(fd)   # scope check before any worker starts (raises NotImplementedError)
    n_total = ((W + 7) // 8) * ((H + 7) // 8)
    perm = np.random.default_rng(rng_seed).permutation(n_total).astype(np.int32)
    # calibrate one core on 4 tiles (256 pixels per batch, the smallest batch a worker sees)
    _, dt = _tiles_worker((fd, cam, W, H, perm[:4], spp, depth, seed))
    per_tile = max(dt / 4, 1e-4)
    n = int(min(n_total, max(procs, seconds * procs / per_tile)))
    ids = np.sort(perm[:n])
    parts = [p for p in np.array_split(ids, procs) if p.size]
    ctx = mp.get_context("spawn")   # fresh interpreters: nothing inherited from a GPU process
    with ctx.Pool(len(parts)) as pool:
        pool.map(abs, range(len(parts)))   # start every worker before the clock
        t0 = time.perf_counter()
        res = pool.map(_tiles_worker, [(fd, cam, W, H, p, spp, depth, seed) for p in parts])
        wall = time.perf_counter() - t0
    return ids, np.concatenate([r[0] for r in res]), wall
