"""While-while traversal of the Cornell BVH4 (octant front-to-back child order, as the LDS kernels'
octant copies) simulated on the CPU for waves of 64 extension rays (round 5, profiles/r05/coherence_sim/):
the leaf-buffering depth (npost: leaves a lane may hold before it stops descending; the kernels' "leaf +
cur" is 2) and the leaf-phase entry / exit thresholds (lb / le, the kernels' PRT_LEAF_BREAK / PRT_LEAF_EXIT),
priced with the per-trip VALU counts of the pooled kernel's ISA (79 per node visit, 73 per triangle test),
and the packed leaf trips of traverse_pk (every held leaf's triangles 64 to a trip).
The greedy collapse stands in for the build's SAH-optimal one (3.44 vs 3.17 node visits per query); at
npost 2 the lane fractions match the GPU lane table (0.463 / 0.269 against 0.444 / 0.294).

    python tools/bvh4_sim.py
"""
import numpy as np, sys, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from tools.coherence_sim import bounce_rays  # noqa: E402
from pyrenderer_amd import scenes
from pyrenderer_amd.io_utils.read_tungsten import read_file
from pyrenderer_amd.flatten import flatten_scene
from pyrenderer_amd._native import Bvh
SENT = 1 << 30

def load(max_leaf=4):
    scene, cam = read_file(scenes.CORNELL)
    flat = flatten_scene(scene)
    nodes, tris, _ = Bvh(flat.tri_v, max_leaf=max_leaf).export()
    refs = nodes[:, 12:14].astype(np.float32).view(np.int32)
    def child(n, s):
        f = nodes[n, 6 * s:6 * s + 6].astype(np.float64)
        return (np.array([f[0], f[2], f[4]]), np.array([f[1], f[3], f[5]]), int(refs[n, s]))
    def area(c):
        d = c[1] - c[0]; return 2 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0])
    # greedy BVH4 collapse
    n4 = []          # list of children lists
    def make(n2):
        ch = [child(n2, 0), child(n2, 1)]
        while len(ch) < 4:
            inner = [i for i, c in enumerate(ch) if c[2] >= 0]
            if not inner: break
            i = max(inner, key=lambda i: area(ch[i]))
            c = ch.pop(i); ch += [child(c[2], 0), child(c[2], 1)]
        me = len(n4); n4.append(None)
        out = []
        for c in ch:
            if c[2] >= 0: out.append((c[0], c[1], make(c[2])))
            else: out.append(c)
        n4[me] = out
        return me
    make(0)
    # octant orders
    orders = []
    for ch in n4:
        o8 = []
        for k in range(8):
            def key(c):
                s = 0.0
                for ax in range(3):
                    s += -c[1][ax] if (k >> ax) & 1 else c[0][ax]
                return s
            o8.append(sorted(range(len(ch)), key=lambda i: (key(ch[i]), i)))
        orders.append(o8)
    T = tris.reshape(-1, 3, 4).astype(np.float64)
    return flat, cam, n4, orders, T

class Sim:
    def __init__(self, n4, orders, T):
        self.n4, self.orders, self.T = n4, orders, T
    def hitbox(self, c, o, inv, tmax):
        t0 = (c[0] - o) * inv; t1 = (c[1] - o) * inv
        tn = max(np.max(np.minimum(t0, t1)), 1e-5); tf = min(np.min(np.maximum(t0, t1)), tmax)
        return tn <= tf
    def tri(self, k, o, d, best):
        v0, e1, e2 = self.T[k, 0, :3], self.T[k, 1, :3], self.T[k, 2, :3]
        c = np.cross(e1, d); det = c @ e2
        if det == 0: return None
        f = 1.0 / det; s = o - v0; q = np.cross(s, e2)
        t, u, v = -f * (q @ e1), -f * (q @ d), f * (c @ s)
        return t if (1e-5 < t < best and u >= 0 and v >= 0 and 1 - u - v >= 0) else None
    def visit(self, j, st):
        o, d, inv, anyq = st['o'][j], st['d'][j], st['inv'][j], st['any'][j]
        k = int(d[0] < 0) | (int(d[1] < 0) << 1) | (int(d[2] < 0) << 2)
        ch = self.n4[st['cur'][j]]
        order = self.orders[st['cur'][j]][k]
        hits = [ch[i][2] for i in order if self.hitbox(ch[i], o, inv, st['best'][j])]
        if anyq: hits = hits[::-1]
        if hits:
            st['cur'][j] = hits[0]
            for r in reversed(hits[1:]): st['stk'][j].append(r)
        else:
            st['cur'][j] = st['stk'][j].pop()

    def wave(self, queries, lb=0, le=8, npost=1, packed=False):
        """Trip counts of one wave: (inner trips, inner lanes, triangle trips, triangle lanes, leaf rounds).
        packed: a leaf round tests the (lane, triangle) pairs of every held leaf 64 to a trip
        (traverse_pk, round 5) against each lane's bound at the round's start."""
        n = len(queries)
        st = {'o': [None]*n, 'd': [None]*n, 'inv': [None]*n, 'best': [0.0]*n, 'any': [False]*n,
              'cur': [SENT]*n, 'leaves': [[] for _ in range(n)], 'stk': [[SENT] for _ in range(n)], 'qi': [0]*n}
        def start(j):
            q = queries[j][st['qi'][j]]; st['qi'][j] += 1
            st['o'][j], st['d'][j], st['best'][j], st['any'][j] = q
            st['inv'][j] = 1.0 / np.where(q[1] == 0, 1e-30, q[1])
            st['cur'][j], st['leaves'][j], st['stk'][j] = 0, [], [SENT]
        def active(j): return not (st['cur'][j] == SENT and not st['leaves'][j])
        wi = li = wl = ll = rounds = 0
        while True:
            for j in range(n):
                if not active(j) and st['qi'][j] < len(queries[j]): start(j)
            if not any(active(j) for j in range(n)): break
            while True:
                lanes = [j for j in range(n) if st['cur'][j] >= 0 and st['cur'][j] != SENT and len(st['leaves'][j]) < npost]
                if not lanes: break
                wi += 1; li += len(lanes)
                for j in lanes:
                    self.visit(j, st)
                    while st['cur'][j] != SENT and st['cur'][j] < 0 and len(st['leaves'][j]) < npost:
                        st['leaves'][j].append(st['cur'][j]); st['cur'][j] = st['stk'][j].pop()
                if sum(1 for j in range(n) if st['cur'][j] >= 0 and st['cur'][j] != SENT and not st['leaves'][j]) <= lb: break
            while True:
                lanes = [j for j in range(n) if st['leaves'][j]]
                if not lanes: break
                rounds += 1
                work = {}
                for j in lanes:
                    tl = []
                    for lf in st['leaves'][j]:
                        v = -lf - 1; tl += list(range(v >> 3, (v >> 3) + (v & 7) + 1))
                    work[j] = tl
                done_any = set()
                if packed:
                    P = sum(len(w) for w in work.values())
                    wl += -(-P // 64); ll += P
                    for j in lanes:
                        b0 = st['best'][j]
                        ts = [t for t in (self.tri(k, st['o'][j], st['d'][j], b0) for k in work[j]) if t is not None]
                        if ts:
                            st['best'][j] = min(ts)
                            if st['any'][j]: done_any.add(j)
                for k in range(0 if packed else max(len(w) for w in work.values())):
                    act = [j for j in lanes if k < len(work[j]) and j not in done_any]
                    if not act: break
                    wl += 1; ll += len(act)
                    for j in act:
                        t = self.tri(work[j][k], st['o'][j], st['d'][j], st['best'][j])
                        if t is not None:
                            st['best'][j] = t
                            if st['any'][j]: done_any.add(j)
                for j in lanes:
                    st['leaves'][j] = []
                    if j in done_any: st['cur'][j] = SENT; continue
                    while st['cur'][j] != SENT and st['cur'][j] < 0 and len(st['leaves'][j]) < npost:
                        st['leaves'][j].append(st['cur'][j]); st['cur'][j] = st['stk'][j].pop()
                if sum(1 for j in range(n) if st['leaves'][j]) <= le: break
        return wi, li, wl, ll, rounds

if __name__ == "__main__":
    flat, cam, n4, orders, T = load()
    print("BVH4 nodes", len(n4))
    sim = Sim(n4, orders, T)
    rng = np.random.default_rng(0)
    O_, D_, B = bounce_rays(flat, cam, 20000, rng)
    perm = rng.permutation(len(O_))[:64 * 150]
    def run(label, X=30, Y=25, **kw):
        """X / Y: extra VALU per packed trip (owner scan, (t, id) reduction) / per packed round (prefix sums)"""
        wi = li = wl = ll = rr = 0
        for g in range(0, len(perm), 64):
            r = sim.wave([[(O_[i], D_[i], 99999.9, False)] for i in perm[g:g + 64]], **kw)
            wi, li, wl, ll, rr = wi + r[0], li + r[1], wl + r[2], ll + r[3], rr + r[4]
        nq = len(perm)
        pk = kw.get("packed", False)
        cost = (wi * 79 + wl * (73 + (X if pk else 0)) + (rr * Y if pk else 0)) / (nq / 64)
        print(f"{label:28s} inner trips/wave {wi/(nq/64):.2f} lanes {li/(64*wi):.3f} | tri trips/wave {wl/(nq/64):.2f} lanes {ll/(64*wl):.3f} | visits/ray {li/nq:.2f} tests/ray {ll/nq:.2f} | VALU/wave {cost:.0f}", flush=True)
    print("---")
    for npost in (2, 3, 4):
        for lb, le in ((0, 8), (4, 8), (8, 8), (0, 16), (8, 16)):
            run(f"npost {npost} lb{lb} le{le}", npost=npost, lb=lb, le=le)
    print("--- packed leaf trips (traverse_pk): 30 extra VALU per trip, 25 per round")
    for npost in (1, 2, 3, 4):
        for lb, le in ((0, 0), (0, 8), (4, 8)):
            run(f"packed npost {npost} lb{lb} le{le}", npost=npost, lb=lb, le=le, packed=True)
