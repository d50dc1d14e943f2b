"""Generate the golden fixtures under tests/golden/ from the reference itself.

FIXTURE-GENERATION ONLY — runs in the build container, never on the GPU box,
never imported by the product.  It executes pyrenderer's own Python source
(`/root/reference`, read-only; bytecode caching disabled) with CPU stand-ins for
the JIT/geometry libraries the image lacks (taichi, taichi_glsl, trimesh, pyrr,
numba, open3d — see `standins/`), and records inputs + outputs as small .npz
vectors.  The reference itself cannot travel; these vectors do.

Usage (from the repo root):
    python tests/golden/gen/make_golden.py scene hits kats trace
    python tests/golden/gen/make_golden.py image --depth 4 --res 32 --spp 256 --procs 6

Fixtures written (all under tests/golden/):
  scene_cornell.npz   per-primitive world vertices/faces/normals/bsdf of
                      media/cornell-box/scene.json as the reference loads it
                      (io_utils/read_tungsten.py:15-46, mathematics/shapes.py:17-57,
                      :119-186), the reference World BVH (accelerators/bvh_taichi.py:111-161)
                      and the camera (core/camera.py:14-36, core/camera_taichi.py:10-39).
  hits_cornell.npz    closest-hit queries answered by World.hit_all
                      (mathematics/intersection_taichi.py:238-291), incl. the 9
                      recorded bounces of test.py:38-57 and shadow-style queries
                      bounded by t_at_light (core/tracing.py:99-102).
  kats.npz            unit known-answer vectors: ray_triangle_hit (:69-91),
                      hit_aabb (bvh_taichi.py:168-190), concentric disk / cosine
                      hemisphere (samplers.py:9-32), rotate_z_to/rotate_vector
                      (mat4_taichi.py:9-60), gen_ray (camera_taichi.py:47-74),
                      hit_sphere (intersection_taichi.py:15-36), reflect / refract /
                      reflectance (bsdf_taichi.py:6-22), Quad.sample_a_point
                      (shapes.py:62-71) and BSDFLambertian.scatter (bsdf.py:29-34).
  trace_cornell.npz   PathTracer.trace (core/tracing.py:116-155) driven through the
                      render() body of main_taichi.py:89-99 with SCRIPTED random
                      streams: per sample the stream, the pixel, the number of
                      draws consumed and the radiance returned.
  mis_cornell.npz     PathTracer.sample_direct_lighting2 (core/tracing.py:57-90), the
                      reference's unused MIS direct-lighting estimator, with scripted
                      streams at camera-ray hit points, and its helpers' unit vectors.
  image_d{D}.npz      statistical reference image: per-pixel mean and standard
                      error of main_taichi.py's render() at res×res, spp, depth D.
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import refload  # noqa: E402

SCENE_JSON = "/root/reference/media/cornell-box/scene.json"


def _load():
    ti = refload.install()
    from io_utils.read_tungsten import read_file
    from mathematics.intersection_taichi import World
    cwd = os.getcwd()
    os.chdir("/root/reference")
    try:
        scene, cam = read_file(SCENE_JSON)
    finally:
        os.chdir(cwd)
    world = World()
    for p in scene.primitives:
        world.add(p)
    world.commit()
    return ti, scene, cam, world


def gen_scene():
    ti, scene, cam, world = _load()
    out = {}
    prims = scene.primitives
    out["n_prim"] = np.int32(len(prims))
    out["prim_type"] = np.array([0 if type(p).__name__ == "Quad" else 1 for p in prims], np.int32)
    nv = [p.vertices.shape[0] for p in prims]
    nf = [p.faces.shape[0] for p in prims]
    out["prim_vert_off"] = np.concatenate([[0], np.cumsum(nv)]).astype(np.int32)
    out["prim_face_off"] = np.concatenate([[0], np.cumsum(nf)]).astype(np.int32)
    out["vertices_f64"] = np.concatenate([p.vertices for p in prims]).astype(np.float64)
    out["vertices_f32"] = np.concatenate([p.vertices_ti.data[:, 0, :] for p in prims]).astype(np.float32)
    out["faces"] = np.concatenate([np.asarray(p.faces, np.int64) for p in prims]).astype(np.int32)
    out["normals"] = np.concatenate([p.normals_ti.data[:, 0, :] for p in prims]).astype(np.float32)
    out["trans_mat"] = np.stack([np.asarray(p.trans_mat, np.float64) for p in prims])
    rho = []
    for p in prims:
        r = p.bsdf.rho
        rho.append(np.array([r, r, r] if np.isscalar(r) else [r[0], r[1], r[2]], np.float32))
    out["rho"] = np.stack(rho)
    out["emit"] = np.array([p.bsdf.emitting_light for p in prims], np.int32)
    out["sided"] = np.array([p.bsdf.sided for p in prims], np.int32)
    out["bounds_min"] = np.stack([np.asarray(p.bounds.min_coord, np.float64) for p in prims])
    out["bounds_max"] = np.stack([np.asarray(p.bounds.max_coord, np.float64) for p in prims])
    b = world.bvh
    out["bvh_obj"] = b.bvh_obj_id.data.astype(np.int32)
    out["bvh_left"] = b.bvh_left_id.data.astype(np.int32)
    out["bvh_right"] = b.bvh_right_id.data.astype(np.int32)
    out["bvh_next"] = b.bvh_next_id.data.astype(np.int32)
    out["bvh_min"] = b.bvh_min.data.astype(np.float32)
    out["bvh_max"] = b.bvh_max.data.astype(np.float32)
    out["cam_view"] = np.asarray(cam.view, np.float64)
    out["cam_iview"] = np.asarray(cam.iview, np.float64)
    tc = cam.convert_to_taichi_camera()
    out["cam_iview_cols"] = np.stack([tc.iview_c1, tc.iview_c2, tc.iview_c3, tc.iview_c4]).astype(np.float32)
    out["cam_sensor_dim"] = np.asarray(tc.sensor_dim, np.float32)
    out["cam_resolution"] = np.asarray(cam.resolution, np.int32)
    np.savez_compressed(os.path.join(OUT, "scene_cornell.npz"), **out)
    print("scene_cornell.npz:", {k: getattr(v, "shape", ()) for k, v in out.items()})


TEST_PY_RAYS = [  # test.py:38-57 — [hit, t, ro, rd, wi, albedo, normal]
    [1, 7.830270, [0.000000, 1.000000, 6.800000], [0.034281, 0.080880, -0.996134], [0.799974, -0.512694, 0.311747], [0.725000, 0.710000, 0.680000], [-0.000000, 0.000000, 1.000000]],
    [1, 0.914496, [0.268427, 1.633309, -1.000000], [0.799974, -0.512694, 0.311747], [-0.944430, -0.165854, -0.283803], [0.140000, 0.450000, 0.091000], [-1.000000, -0.000000, -0.000000]],
    [1, 1.004540, [1.000000, 1.164452, -0.714908], [-0.944430, -0.165854, -0.283803], [-0.539883, -0.658663, 0.524109], [0.725000, 0.710000, 0.680000], [-0.000000, 0.000000, 1.000000]],
    [1, 0.766014, [0.051282, 0.997845, -1.000000], [-0.539883, -0.658663, 0.524109], [-0.039377, 0.827128, -0.560632], [0.725000, 0.710000, 0.680000], [-0.328669, 0.000000, -0.944445]],
    [1, 0.716111, [-0.362276, 0.493300, -0.598526], [-0.039377, 0.827128, -0.560632], [0.688579, -0.690442, 0.221697], [0.725000, 0.710000, 0.680000], [-0.000000, 0.000000, 1.000000]],
    [1, 1.572349, [-0.390474, 1.085616, -1.000000], [0.688579, -0.690442, 0.221697], [0.631949, 0.704407, -0.323189], [0.725000, 0.710000, 0.680000], [-0.000000, 1.000000, -0.000000]],
    [1, 0.487045, [0.692212, 0.000000, -0.651414], [0.631949, 0.704407, -0.323189], [-0.074693, -0.669229, 0.739292], [0.140000, 0.450000, 0.091000], [-1.000000, -0.000000, -0.000000]],
    [1, 0.512646, [1.000000, 0.343078, -0.808822], [-0.074693, -0.669229, 0.739292], [0.324842, 0.923928, -0.202077], [0.725000, 0.710000, 0.680000], [-0.000000, 1.000000, -0.000000]],
    [1, 0.117876, [0.961709, -0.000000, -0.429826], [0.324842, 0.923928, -0.202077], [-0.052710, -0.073551, 0.995898], [0.140000, 0.450000, 0.091000], [-1.000000, -0.000000, -0.000000]],
]


def _unit(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def gen_hits(n_random=1500, n_shadow=1000, n_axis=200):
    ti, scene, cam, world = _load()
    rng = np.random.default_rng(20241015)
    ti.seed_random(7)
    tc = cam.convert_to_taichi_camera()
    ro_l, rd_l, t0_l, t1_l, kind = [], [], [], [], []
    for row in TEST_PY_RAYS:
        ro_l.append(row[2]); rd_l.append(row[3]); t0_l.append(1e-5); t1_l.append(99999.9); kind.append(0)
    for _ in range(300):  # camera rays (main_taichi.py:93-95)
        u, v = rng.random(2).astype(np.float32)
        o, d = tc.gen_ray(np.float32(u), np.float32(v))
        ro_l.append(o); rd_l.append(d); t0_l.append(1e-5); t1_l.append(99999.9); kind.append(1)
    org = np.stack([rng.uniform(-1, 1, n_random), rng.uniform(0, 2, n_random), rng.uniform(-1, 1, n_random)], 1)
    dirs = _unit(rng, n_random)
    for o, d in zip(org.astype(np.float32), dirs):
        ro_l.append(o); rd_l.append(d); t0_l.append(1e-5); t1_l.append(99999.9); kind.append(2)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    for k in range(n_axis):
        o = np.array([rng.uniform(-0.99, 0.99), rng.uniform(0.01, 1.99), rng.uniform(-0.99, 0.99)], np.float32)
        ro_l.append(o); rd_l.append(axes[k % 6]); t0_l.append(1e-5); t1_l.append(99999.9); kind.append(3)
    # shadow-style queries: from a surface point toward a point on the light,
    # bounded by t_at_light exactly as core/tracing.py:97-102 computes it.
    light = [p for p in scene.primitives if p.bsdf.emitting_light][0]
    lv = light.vertices_ti.data[:, 0, :]
    lf = light.faces_ti.data[:, 0, :]
    made = 0
    while made < n_shadow:
        o = np.array([rng.uniform(-1, 1), rng.uniform(0, 2), rng.uniform(-1, 1)], np.float32)
        d = _unit(rng, 1)[0]
        h = world.hit_all(ti.Vec(o), ti.Vec(d), 0.00001, 99999.9)
        if not h[0]:
            continue
        p = ti.Vec(h[2])
        f = int(rng.integers(0, 2))
        uu = np.sqrt(np.float32(rng.random()))
        vv = np.float32(rng.random())
        a = uu * (1 - vv)
        b = uu * vv
        v0, v1, v2 = lf[f]
        p2 = a * ti.Vec(lv[v0]) + b * ti.Vec(lv[v1]) + (np.float32(1.0) - a - b) * ti.Vec(lv[v2])
        from taichi_glsl.vector import normalize
        w = normalize(p2 - p)
        t_at = (p2[0] - p[0]) / w[0]
        ro_l.append(np.asarray(p, np.float32)); rd_l.append(np.asarray(w, np.float32))
        t0_l.append(1e-5); t1_l.append(t_at); kind.append(4)
        made += 1
    n = len(ro_l)
    ro = np.asarray(ro_l, np.float32)
    rd = np.asarray(rd_l, np.float32)
    t0 = np.asarray(t0_l, np.float32)
    t1 = np.asarray(t1_l, np.float32)
    hit = np.zeros(n, np.int32)
    t = np.zeros(n, np.float32)
    nrm = np.zeros((n, 3), np.float32)
    emit = np.zeros(n, np.int32)
    rho = np.zeros((n, 3), np.float32)
    for i in range(n):
        h = world.hit_all(ti.Vec(ro[i]), ti.Vec(rd[i]), np.float32(t0[i]), np.float32(t1[i]))
        hit[i] = int(bool(h[0]))
        t[i] = h[1]
        nrm[i] = h[3]
        emit[i] = int(h[4])
        rho[i] = h[5]
    np.savez_compressed(os.path.join(OUT, "hits_cornell.npz"), ro=ro, rd=rd, tmin=t0, tmax=t1, kind=np.asarray(kind, np.int32),
                        hit=hit, t=t, normal=nrm, emit=emit, rho=rho,
                        test_py=np.array([[r[1]] + r[2] + r[3] + r[4] + r[5] + r[6] for r in TEST_PY_RAYS], np.float64))
    print("hits_cornell.npz:", n, "queries;", hit.sum(), "hits;", (kind == np.array(4)).sum() if False else sum(1 for k in kind if k == 4), "shadow")


def gen_kats():
    ti, scene, cam, world = _load()
    from mathematics.intersection_taichi import ray_triangle_hit, hit_sphere
    from mathematics import samplers as S
    from mathematics import mat4_taichi as M
    from core import bsdf_taichi as BT
    from core.bsdf import BSDFLambertian
    rng = np.random.default_rng(99)
    out = {}
    # --- ray_triangle_hit ---
    n = 3000
    v0 = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    v1 = (v0 + rng.uniform(-1, 1, (n, 3))).astype(np.float32)
    v2 = (v0 + rng.uniform(-1, 1, (n, 3))).astype(np.float32)
    ro = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    bary = rng.uniform(-0.2, 1.2, (n, 2))
    target = v0 + bary[:, :1] * (v1 - v0) + bary[:, 1:] * (v2 - v0)
    rd = (target - ro)
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    rd[:200] = _unit(rng, 200)                        # arbitrary directions
    rd[200:260] = np.cross(v1[200:260] - v0[200:260], v2[200:260] - v0[200:260]) * 0 + (v1[200:260] - v0[200:260])  # parallel (det==0)
    v2[260:300] = v1[260:300]                         # degenerate triangles
    t0 = np.full(n, 1e-5, np.float32)
    t1 = np.full(n, 99999.9, np.float32)
    t1[300:600] = rng.uniform(0.0, 3.0, 300).astype(np.float32)
    hit = np.zeros(n, np.int32)
    tt = np.zeros(n, np.float32)
    for i in range(n):
        h, t = ray_triangle_hit(ti.Vec(v0[i]), ti.Vec(v1[i]), ti.Vec(v2[i]), ti.Vec(ro[i]), ti.Vec(rd[i]), t0[i], t1[i])
        hit[i] = h
        tt[i] = t
    out.update(tri_v0=v0, tri_v1=v1, tri_v2=v2, tri_ro=ro, tri_rd=rd, tri_t0=t0, tri_t1=t1, tri_hit=hit, tri_t=tt)
    # --- hit_aabb on the reference World BVH nodes + random boxes ---
    b = world.bvh
    nb = 2000
    idx = rng.integers(0, b.bvh_min.data.shape[0], nb)
    bro = np.stack([rng.uniform(-1.5, 1.5, nb), rng.uniform(-0.5, 2.5, nb), rng.uniform(-1.5, 7.0, nb)], 1).astype(np.float32)
    brd = _unit(rng, nb)
    brd[:150, rng.integers(0, 3, 150)] = 0.0          # zero direction components (slab division by 0)
    brd[150:200] = np.array([0, 0, -1], np.float32)
    bt0 = np.full(nb, 1e-5, np.float32)
    bt1 = np.where(rng.random(nb) < 0.3, rng.uniform(0, 5, nb), 99999.9).astype(np.float32)
    bres = np.zeros(nb, np.int32)
    for i in range(nb):
        bres[i] = b.hit_aabb(int(idx[i]), ti.Vec(bro[i]), ti.Vec(brd[i]), bt0[i], bt1[i])
    out.update(aabb_node=idx.astype(np.int32), aabb_min=b.bvh_min.data[idx].astype(np.float32),
               aabb_max=b.bvh_max.data[idx].astype(np.float32), aabb_ro=bro, aabb_rd=brd, aabb_t0=bt0,
               aabb_t1=bt1, aabb_hit=bres)
    # --- samplers (Taichi versions, samplers.py:9-32) ---
    ns = 2000
    u = rng.random((ns, 2)).astype(np.float32)
    u[:5] = np.array([[0.5, 0.5], [0.25, 0.25], [0.75, 0.25], [0.0, 0.5], [0.5, 0.0]], np.float32)
    disk = np.zeros((ns, 2), np.float32)
    hemi = np.zeros((ns, 3), np.float32)
    for i in range(ns):
        disk[i] = S.concentric_sample_disk(ti.Vec(u[i]))
        hemi[i] = S.cosine_sample_hemisphere(ti.Vec(u[i]))
    out.update(smp_u=u, smp_disk=disk, smp_hemi=hemi)
    # --- frames (mat4_taichi.py:9-60) ---
    nf = 1000
    nrm = _unit(rng, nf)
    nrm[:4] = np.array([[0, 1, 0], [0, -1, 0], [1, 0, 0], [0, 0, -1]], np.float32)
    nrm[4:4 + len(scene.primitives[0].normals_ti.data)] = 0
    allnormals = np.concatenate([p.normals_ti.data[:, 0, :] for p in scene.primitives])
    nrm[4:4 + allnormals.shape[0]] = allnormals
    nrm[4 + allnormals.shape[0]:4 + 2 * allnormals.shape[0]] = -allnormals
    vec = hemi[:nf]
    rows = np.zeros((nf, 3, 3), np.float32)
    rot = np.zeros((nf, 3), np.float32)
    for i in range(nf):
        r1, r2, r3, r4 = M.rotate_z_to(ti.Vec(nrm[i]))
        rows[i] = np.stack([r1[:3], r2[:3], r3[:3]])
        rot[i] = M.rotate_vector(r1, r2, r3, ti.Vec(vec[i]))
    out.update(frm_n=nrm, frm_v=vec, frm_rows=rows, frm_out=rot)
    # --- camera gen_ray (camera_taichi.py:47-74) ---
    tc = cam.convert_to_taichi_camera()
    nc = 1000
    cu = rng.random((nc, 2)).astype(np.float32)
    co = np.zeros((nc, 3), np.float32)
    cd = np.zeros((nc, 3), np.float32)
    for i in range(nc):
        o, d = tc.gen_ray(cu[i, 0], cu[i, 1])
        co[i] = o
        cd[i] = d
    out.update(cam_uv=cu, cam_o=co, cam_d=cd)
    # --- hit_sphere (intersection_taichi.py:15-36) ---
    nsph = 2000
    sc = rng.uniform(-1, 1, (nsph, 3)).astype(np.float32)
    sr = rng.uniform(0.05, 1.0, nsph).astype(np.float32)
    so = rng.uniform(-3, 3, (nsph, 3)).astype(np.float32)
    aim = sc + rng.normal(0, 0.7, (nsph, 3))
    sd = aim - so
    sd = (sd / np.linalg.norm(sd, axis=1, keepdims=True)).astype(np.float32)
    so[:100] = sc[:100]                              # origin at centre: far root
    st0 = np.full(nsph, 1e-5, np.float32)
    st1 = np.where(rng.random(nsph) < 0.3, rng.uniform(0, 4, nsph), 99999.9).astype(np.float32)
    sh = np.zeros(nsph, np.int32)
    sroot = np.zeros(nsph, np.float32)
    for i in range(nsph):
        h, r = hit_sphere(ti.Vec(sc[i]), sr[i], ti.Vec(so[i]), ti.Vec(sd[i]), st0[i], st1[i])
        sh[i] = int(bool(h))
        sroot[i] = r
    out.update(sph_c=sc, sph_r=sr, sph_o=so, sph_d=sd, sph_t0=st0, sph_t1=st1, sph_hit=sh, sph_root=sroot)
    # --- reflect / refract / reflectance (bsdf_taichi.py:6-22) ---
    nr = 1000
    rv = _unit(rng, nr)
    rn = _unit(rng, nr)
    flip = np.sum(rv * rn, 1) > 0
    rn[flip] = -rn[flip]                              # incident against the normal
    eta = rng.uniform(0.4, 2.5, nr).astype(np.float32)
    cosv = rng.random(nr).astype(np.float32)
    refl = np.zeros((nr, 3), np.float32)
    refr = np.zeros((nr, 3), np.float32)
    schl = np.zeros(nr, np.float32)
    for i in range(nr):
        refl[i] = BT.reflect(ti.Vec(rv[i]), ti.Vec(rn[i]))
        refr[i] = BT.refract(ti.Vec(rv[i]), ti.Vec(rn[i]), eta[i])
        schl[i] = BT.reflectance(cosv[i], eta[i])
    out.update(rr_v=rv, rr_n=rn, rr_eta=eta, rr_cos=cosv, rr_reflect=refl, rr_refract=refr, rr_schlick=schl)
    # --- Quad.sample_a_point on the light (shapes.py:62-71), scripted draws ---
    light = [p for p in scene.primitives if p.bsdf.emitting_light][0]
    nl = 1000
    draws = rng.random((nl, 3)).astype(np.float32)
    lp = np.zeros((nl, 3), np.float32)
    ln = np.zeros((nl, 3), np.float32)
    le = np.zeros((nl, 3), np.float32)
    for i in range(nl):
        ti.script_random(draws[i])
        p, nn, e = light.sample_a_point()
        lp[i] = p
        ln[i] = nn
        le[i] = e
    ti.script_random(None)
    out.update(light_draws=draws, light_p=lp, light_n=ln, light_e=le)
    # --- BSDFLambertian.scatter (bsdf.py:29-34) + Quad.hit frame rotation ---
    lam = BSDFLambertian({"albedo": [0.725, 0.71, 0.68]})
    nl2 = 500
    d2 = rng.random((nl2, 2)).astype(np.float32)
    wl = np.zeros((nl2, 3), np.float32)
    pl = np.zeros(nl2, np.float32)
    for i in range(nl2):
        ti.script_random(d2[i])
        wi, att, pdf = lam.scatter(ti.Vec([0, 0, -1]))
        wl[i] = wi
        pl[i] = pdf
    ti.script_random(None)
    out.update(lam_draws=d2, lam_wi=wl, lam_pdf=pl)
    np.savez_compressed(os.path.join(OUT, "kats.npz"), **out)
    print("kats.npz:", len(out), "arrays")


def _render_sample(ti, tc, tracer, x, y, w, h, depth):
    """main_taichi.py:89-99 — one sample of render() for pixel (x, y)."""
    u = (x + ti.random()) / (w - 1)
    v = (y + ti.random()) / (h - 1)
    o, d = tc.gen_ray(u, v)
    return tracer.trace(o, d, depth, x, y)


def gen_trace(n_samples=1500, depths=(4, 8), stream_len=256, res=512):
    ti, scene, cam, world = _load()
    from core.tracing import PathTracer
    tc = cam.convert_to_taichi_camera()
    rng = np.random.default_rng(4242)
    out = {}
    for depth in depths:
        tracer = PathTracer(world, depth, res, res)
        streams = rng.random((n_samples, stream_len)).astype(np.float32)
        px = rng.integers(0, res, (n_samples, 2)).astype(np.int32)
        col = np.zeros((n_samples, 3), np.float32)
        used = np.zeros(n_samples, np.int32)
        for i in range(n_samples):
            ti.script_random(streams[i])
            col[i] = _render_sample(ti, tc, tracer, int(px[i, 0]), int(px[i, 1]), res, res, depth)
            used[i] = ti.script_consumed()
        ti.script_random(None)
        out[f"d{depth}_streams"] = streams
        out[f"d{depth}_pixel"] = px
        out[f"d{depth}_color"] = col
        out[f"d{depth}_used"] = used
        print(f"trace depth {depth}: mean {col.mean(0)}, draws/sample {used.mean():.1f} (max {used.max()})")
    out["res"] = np.int32(res)
    np.savez_compressed(os.path.join(OUT, "trace_cornell.npz"), **out)


def gen_mis(n=1500, stream_len=64, res=512):
    """mis_cornell.npz: the reference's unused MIS direct-lighting estimator
    PathTracer.sample_direct_lighting2 (core/tracing.py:57-90) at surface points hit by
    camera rays, replayed with SCRIPTED random streams (inputs, stream, draws consumed,
    result), plus unit vectors of its helpers mis_power_heuristic / compute_area_light_pdf
    / compute_brdf_pdf / dot_or_zero (core/tracing.py:12-39)."""
    ti, scene, cam, world = _load()
    from core.tracing import (PathTracer, compute_area_light_pdf, compute_brdf_pdf, dot_or_zero,
                              mis_power_heuristic)
    tc = cam.convert_to_taichi_camera()
    tracer = PathTracer(world, 8, res, res)
    rng = np.random.default_rng(777)
    pts, nrms, rhos, streams, outs, used = [], [], [], [], [], []
    while len(pts) < n:
        x, y = (int(v) for v in rng.integers(0, res, 2))
        ti.script_random(rng.random(64).astype(np.float32))
        u = (x + ti.random()) / (res - 1)
        v = (y + ti.random()) / (res - 1)
        o, d = tc.gen_ray(u, v)
        hit, t, p, nrm, emissive, att, _, _ = world.hit_all(o, d, 0.00001, 99999.9)
        ti.script_random(None)
        if not hit or emissive > 0:
            continue
        st = rng.random(stream_len).astype(np.float32)
        ti.script_random(st)
        li = tracer.sample_direct_lighting2(p, nrm, att)
        used.append(ti.script_consumed())
        ti.script_random(None)
        pts.append(np.asarray(p, np.float32)); nrms.append(np.asarray(nrm, np.float32))
        rhos.append(np.asarray(att, np.float32)); streams.append(st); outs.append(np.asarray(li, np.float32))
    out = dict(p=np.stack(pts), n=np.stack(nrms), rho=np.stack(rhos), streams=np.stack(streams),
               direct=np.stack(outs), used=np.asarray(used, np.int32))
    k = 400
    pf = (rng.random(k) * 4).astype(np.float32)
    pg = (rng.random(k) * 4).astype(np.float32)
    out["pw_f"], out["pw_g"] = pf, pg
    out["pw_out"] = np.array([mis_power_heuristic(pf[i], pg[i]) for i in range(k)], np.float32)
    dirs = rng.normal(size=(k, 3)).astype(np.float32)
    dirs = (dirs / np.linalg.norm(dirs, axis=1, keepdims=True)).astype(np.float32)
    n2 = rng.normal(size=(k, 3)).astype(np.float32)
    n2 = (n2 / np.linalg.norm(n2, axis=1, keepdims=True)).astype(np.float32)
    tl = (rng.random(k) * 5).astype(np.float32)
    out["ap_t"], out["ap_d"], out["ap_n"] = tl, dirs, n2
    out["ap_out"] = np.array([compute_area_light_pdf(tl[i], ti.Vec(dirs[i]), ti.Vec(n2[i]), 1.0)
                              for i in range(k)], np.float32)
    out["bp_out"] = np.array([compute_brdf_pdf(ti.Vec(n2[i]), ti.Vec(dirs[i])) for i in range(k)], np.float32)
    out["dz_out"] = np.array([dot_or_zero(ti.Vec(n2[i]), ti.Vec(dirs[i])) for i in range(k)], np.float32)
    np.savez_compressed(os.path.join(OUT, "mis_cornell.npz"), **out)
    nz = (np.abs(out["direct"]).sum(1) > 0).mean()
    print(f"mis_cornell.npz: {n} points, non-zero direct {nz:.2f}, draws {np.mean(used):.1f}")


def _image_worker(args):
    rows, res, spp, depth, seed = args
    ti, scene, cam, world = _load()
    from core.tracing import PathTracer
    tc = cam.convert_to_taichi_camera()
    tracer = PathTracer(world, depth, res, res)
    ti.seed_random(seed)
    s1 = np.zeros((len(rows), res, 3), np.float64)
    s2 = np.zeros((len(rows), res, 3), np.float64)
    for k, y in enumerate(rows):
        for x in range(res):
            for _ in range(spp):
                c = np.asarray(_render_sample(ti, tc, tracer, x, y, res, res, depth), np.float64)
                s1[k, x] += c
                s2[k, x] += c * c
    return rows, s1, s2


def gen_image(depth, res, spp, procs):
    jobs = []
    for r in range(res):
        jobs.append(([r], res, spp, depth, 1000 * depth + r))
    t0 = time.time()
    s1 = np.zeros((res, res, 3))
    s2 = np.zeros((res, res, 3))
    with mp.get_context("fork").Pool(procs) as pool:
        for rows, a, b in pool.imap_unordered(_image_worker, jobs):
            for k, y in enumerate(rows):
                s1[y] = a[k]
                s2[y] = b[k]
            print(f"  row {rows[0]} done ({time.time() - t0:.0f}s)", flush=True)
    mean = s1 / spp
    var = np.maximum(s2 / spp - mean * mean, 0.0) * spp / (spp - 1)
    se = np.sqrt(var / spp)
    # stored [x][y] like the reference's pixels field (main_taichi.py:25,89)
    np.savez_compressed(os.path.join(OUT, f"image_d{depth}.npz"), mean=mean.transpose(1, 0, 2).astype(np.float32),
                        se=se.transpose(1, 0, 2).astype(np.float32), spp=np.int32(spp), depth=np.int32(depth),
                        res=np.int32(res))
    print(f"image_d{depth}.npz: mean {mean.mean((0, 1))}, {time.time() - t0:.0f}s")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="+", choices=["scene", "hits", "kats", "trace", "mis", "image"])
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--res", type=int, default=32)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--procs", type=int, default=6)
    a = ap.parse_args()
    for w in a.what:
        if w == "scene":
            gen_scene()
        elif w == "hits":
            gen_hits()
        elif w == "kats":
            gen_kats()
        elif w == "trace":
            gen_trace()
        elif w == "mis":
            gen_mis()
        elif w == "image":
            gen_image(a.depth, a.res, a.spp, a.procs)
