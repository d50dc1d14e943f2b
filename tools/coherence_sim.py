"""Ray-grouping schedules for the LDS-resident traversal, priced on the CPU (round 5; results in
profiles/r05/coherence_sim/results.txt).

A Python model of the kernels' while-while traversal (Aila & Laine 2009: descend until every lane
holds a leaf, test leaves until <= 8 lanes hold one) over the Cornell BVH2, run on waves of 64 rays,
counts wave-level trips and the lanes active in them.  For randomly grouped rays it reproduces the GPU
lane table (tools/lane_table.py: 0.44 of the lanes in inner-node visits, 0.29 in triangle tests), so it
prices schedules before any kernel is written:
  * rays sorted by direction octant (and origin cell) inside a window of 256 — the block's pooled
    extension rays that VERDICT r04 item 1 proposed: +1 % lanes;
  * a lane running its extension query and then its own shadow ray in one loop (no pool, no barrier):
    fewer lanes than the two-phase pool;
  * several extension queries chained per lane.

    python tools/coherence_sim.py [--waves 300]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SENT = 1 << 30


class Model:
    def __init__(self, flat):
        from pyrenderer_amd._native import Bvh
        nodes, tris, _ = Bvh(flat.tri_v).export()
        self.nodes = nodes.astype(np.float64)
        self.refs = nodes[:, 12:14].astype(np.float32).view(np.int32)
        self.T = tris.reshape(-1, 3, 4).astype(np.float64)

    def box(self, n, side, o, inv, tmax):
        f = self.nodes[n, 6 * side:6 * side + 6]
        lo = np.array([f[0], f[2], f[4]])
        hi = np.array([f[1], f[3], f[5]])
        t0, t1 = (lo - o) * inv, (hi - o) * inv
        tn = max(np.max(np.minimum(t0, t1)), 1e-5)
        tf = min(np.min(np.maximum(t0, t1)), tmax)
        return tn <= tf, tn

    def tri(self, k, o, d, best):
        v0, e1, e2 = self.T[k, 0, :3], self.T[k, 1, :3], self.T[k, 2, :3]
        c = np.cross(e1, d)
        det = c @ e2
        if det == 0:
            return None
        f = 1.0 / det
        s = o - v0
        q = np.cross(s, e2)
        t, u, v = -f * (q @ e1), -f * (q @ d), f * (c @ s)
        return t if (1e-5 < t < best and u >= 0 and v >= 0 and 1 - u - v >= 0) else None

    def wave(self, queries, lb=0, le=8):
        """queries[j]: (o, d, t_max, any-hit) tuples run one after another by lane j in ONE while-while
        loop (the next one taken at the top of the next round).  Returns (inner wave trips, inner lane
        trips, triangle wave trips, triangle lane trips)."""
        n = len(queries)
        qi = [0] * n
        o, d, inv, best, anyq = [None] * n, [None] * n, [None] * n, [0.0] * n, [False] * n
        cur, leaf, stk = [SENT] * n, [0] * n, [[SENT] for _ in range(n)]

        def start(j):
            o[j], d[j], best[j], anyq[j] = queries[j][qi[j]]
            qi[j] += 1
            inv[j] = 1.0 / np.where(d[j] == 0, 1e-30, d[j])
            cur[j], leaf[j], stk[j] = 0, 0, [SENT]

        def active(j):
            return not (cur[j] == SENT and leaf[j] >= 0)

        wi = li = wl = ll = 0
        while True:
            for j in range(n):
                if not active(j) and qi[j] < len(queries[j]):
                    start(j)
            if not any(active(j) for j in range(n)):
                break
            while True:
                lanes = [j for j in range(n) if cur[j] >= 0 and cur[j] != SENT]
                if not lanes:
                    break
                wi += 1
                li += len(lanes)
                for j in lanes:
                    nd, h = cur[j], []
                    for s in (0, 1):
                        ok, tn = self.box(nd, s, o[j], inv[j], best[j])
                        if ok:
                            h.append((tn, self.refs[nd, s]))
                    h.sort(key=lambda x: x[0], reverse=anyq[j])
                    if len(h) == 2:
                        stk[j].append(h[1][1])
                        cur[j] = h[0][1]
                    elif len(h) == 1:
                        cur[j] = h[0][1]
                    else:
                        cur[j] = stk[j].pop()
                    if cur[j] != SENT and cur[j] < 0 and leaf[j] >= 0:
                        leaf[j] = cur[j]
                        cur[j] = stk[j].pop()
                if sum(1 for j in range(n) if cur[j] >= 0 and cur[j] != SENT and leaf[j] >= 0) <= lb:
                    break
            while True:
                lanes = [j for j in range(n) if leaf[j] < 0]
                if not lanes:
                    break
                cnts = {j: ((-leaf[j] - 1) >> 3, ((-leaf[j] - 1) & 7) + 1) for j in lanes}
                hit_any = set()
                for k in range(max(c for _, c in cnts.values())):
                    act = [j for j in lanes if k < cnts[j][1] and j not in hit_any]
                    if not act:
                        break
                    wl += 1
                    ll += len(act)
                    for j in act:
                        t = self.tri(cnts[j][0] + k, o[j], d[j], best[j])
                        if t is not None:
                            best[j] = t
                            if anyq[j]:
                                hit_any.add(j)
                for j in lanes:
                    if j in hit_any:
                        cur[j], leaf[j] = SENT, 0
                        continue
                    leaf[j] = cur[j] if (cur[j] != SENT and cur[j] < 0) else 0
                    if leaf[j] < 0:
                        cur[j] = stk[j].pop()
                if sum(1 for j in range(n) if leaf[j] < 0) <= le:
                    break
        return wi, li, wl, ll


def bounce_rays(flat, cam, n, rng):
    """Camera rays and three cosine bounces (closest hits by the C oracle): origins and directions
    per bounce level."""
    from oracle import oracle as O
    osc = O.OracleScene.from_flat(flat)
    tv = flat.tri_v.reshape(-1, 3, 3).astype(np.float64)
    o, d = cam.convert_to_taichi_camera().gen_ray(rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32))
    out = []
    for b in range(4):
        out.append((o.astype(np.float64), d.astype(np.float64), np.full(n, b)))
        hit, t, tri, _ = osc.closest(o, d, np.float32(1e-5), np.float32(99999.9))
        ok = hit > 0
        p = o + d * t[:, None]
        tr = tv[np.maximum(tri, 0)]
        nn = np.cross(tr[:, 1] - tr[:, 0], tr[:, 2] - tr[:, 0])
        nn /= np.linalg.norm(nn, axis=1)[:, None]
        nn = np.where((np.sum(nn * d, axis=1) > 0)[:, None], -nn, nn)
        phi, r2 = 2 * np.pi * rng.random(n), rng.random(n)
        lx, ly, lz = np.sqrt(r2) * np.cos(phi), np.sqrt(r2) * np.sin(phi), np.sqrt(1 - r2)
        a = np.where(np.abs(nn[:, 0:1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
        tx = np.cross(nn, a)
        tx /= np.linalg.norm(tx, axis=1)[:, None]
        ty = np.cross(nn, tx)
        dn = tx * lx[:, None] + ty * ly[:, None] + nn * lz[:, None]
        o = np.where(ok[:, None], p, o).astype(np.float32)
        d = np.where(ok[:, None], dn, d).astype(np.float32)
    return [np.concatenate(x) for x in zip(*out)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=300)
    ap.add_argument("--rays", type=int, default=40000)
    a = ap.parse_args()
    from pyrenderer_amd import scenes
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(scenes.CORNELL)
    flat = flatten_scene(scene)
    m = Model(flat)
    rng = np.random.default_rng(0)
    O_, D_, B = bounce_rays(flat, cam, a.rays, rng)
    M = 64 * a.waves
    perm = rng.permutation(len(O_))[:M]

    def report(label, groups):
        wi = li = wl = ll = 0
        for g in groups:
            r = m.wave([[(O_[i], D_[i], 99999.9, False)] for i in g])
            wi, li, wl, ll = wi + r[0], li + r[1], wl + r[2], ll + r[3]
        print(f"{label:34s}: inner lanes {li / (64 * wi):.3f}, triangle-test lanes {ll / (64 * wl):.3f}", flush=True)

    octant = (D_[:, 0] < 0) * 1 + (D_[:, 1] < 0) * 2 + (D_[:, 2] < 0) * 4
    cell = np.floor((O_ + 1.2) / 0.6).astype(int) @ np.array([1, 8, 64])

    def sorted_windows(key, w):
        gs = []
        for i in range(0, M, w):
            win = perm[i:i + w]
            win = win[np.argsort(key[win], kind="stable")]
            gs += [win[k:k + 64] for k in range(0, len(win), 64)]
        return gs
    report("random", [perm[i:i + 64] for i in range(0, M, 64)])
    report("octant-sorted / 256", sorted_windows(octant, 256))
    report("octant + origin cell / 256", sorted_windows(octant * 4096 + cell, 256))
    report("octant-sorted / 1024", sorted_windows(octant, 1024))
    report("octant + origin cell / 4096", sorted_windows(octant * 4096 + cell, 4096))


if __name__ == "__main__":
    main()
