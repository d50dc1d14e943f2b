/*
 * prt_oracle.c — CPU restatement of pyrenderer's path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
 * (ctypes, oracle/_build/libprt_oracle.so).  The product path (pyrenderer_amd/)
 * never links or calls it and fails loudly when its HIP library is missing.
 *
 * What it restates (reference @ /root/reference, file:line):
 *   ray_triangle_hit .............. mathematics/intersection_taichi.py:69-91
 *   hit_sphere .................... mathematics/intersection_taichi.py:15-36
 *   World.hit_all ................. mathematics/intersection_taichi.py:238-291
 *   BVH build / hit_aabb .......... accelerators/bvh_taichi.py:58-195
 *   Quad.hit / Cube.hit ........... mathematics/shapes.py:76-110, 205-239
 *   Quad.sample_a_point ........... mathematics/shapes.py:62-71
 *   World.sample_a_light .......... mathematics/intersection_taichi.py:194-207
 *   concentric disk / cos-hemi .... mathematics/samplers.py:9-32
 *   rotate_to/rotate_z_to/rotate_vector  mathematics/mat4_taichi.py:9-60
 *   BSDFLambertian / BSDFLight .... core/bsdf.py:18-65
 *   reflect/refract/reflectance ... core/bsdf_taichi.py:6-22
 *   CameraTaichi.gen_ray .......... core/camera_taichi.py:47-74
 *   PathTracer.trace .............. core/tracing.py:116-155
 *   sample_direct_lighting ........ core/tracing.py:92-108
 *   render() sample body .......... main_taichi.py:89-99
 *
 * Arithmetic: IEEE f32, compiled with -ffp-contract=off and no fast-math, each
 * expression evaluated in the reference's left-to-right order.  Two
 * deliberate, documented deviations shared with the HIP kernel:
 *   - random numbers come from a counter-keyed PCG stream (Taichi's stateful
 *     ti.random() is not reproducible), drawn once per closest hit rather than
 *     once per candidate primitive (distribution-neutral), unless the caller
 *     replays a scripted stream in reference order (or_trace_scripted);
 *   - cos/sin in the concentric map use fixed minimax polynomials (identical
 *     bits on CPU and GPU); cos(pi/2 - a) is evaluated as sin(a).
 * Closest-hit ties (equal t) resolve to the lower triangle index in the
 * brute-force backend; the reference-structure backend keeps the reference's
 * first-found-wins order.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_API __attribute__((visibility("default")))

/* mathematics/constants.py:3-16 (cast to f32 as Taichi's default_fp does) */
static const float kInvPi = 0.31830988618379067154f;
static const float kPiOver4 = 0.78539816339744830961f;
static const float kTMin = 0.00001f;     /* core/tracing.py:127 */
static const float kTMax = 99999.9f;     /* core/tracing.py:127 */

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
/* Taichi Matrix.dot = left-to-right sum of products */
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* taichi_glsl normalize(v) = v / length(v) */
static inline v3 normalize(v3 a) {
    float l = sqrtf(dot(a, a));
    return mk(a.x / l, a.y / l, a.z / l);
}
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline void st3(float* p, v3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

/* ---------------------------------------------------------------- RNG spec */
/* PCG-RXS-M-XS 32 output permutation; LCG step 747796405u, 2891336453u.   */
static inline uint32_t pcg_permute(uint32_t s) {
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
static inline uint32_t pcg_hash(uint32_t v) { return pcg_permute(v * 747796405u + 2891336453u); }

typedef struct {
    uint32_t state;
    const float* script;   /* scripted stream (reference order) or NULL */
    int script_len;
    int pos;
    int overflow;
} Rng;

static inline uint32_t rng_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    uint32_t h = pcg_hash((uint32_t)seed);
    h = pcg_hash(h ^ (uint32_t)(seed >> 32) ^ pixel);
    return pcg_hash(h + sample);
}

static inline float rng_next(Rng* r) {
    if (r->script) {
        if (r->pos >= r->script_len) { r->overflow = 1; return 0.0f; }
        return r->script[r->pos++];
    }
    r->state = r->state * 747796405u + 2891336453u;
    r->pos++;
    return (float)(pcg_permute(r->state) >> 8) * 0x1p-24f;
}

/* taichi_glsl randInt(a, b), inclusive of b (assumption) */
static inline int rng_int(Rng* r, int a, int b) {
    float u = rng_next(r);
    int k = (int)floorf(u * (float)(b - a + 1));
    if (k > b - a) k = b - a;
    return a + k;
}

/* --------------------------------------------------- sin/cos on [-pi/4,pi/4] */
static inline float poly_sin(float x) {
    float z = x * x;
    return ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x + x;
}
static inline float poly_cos(float x) {
    float z = x * x;
    return ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
           - 0.5f * z + 1.0f;
}

/* ------------------------------------------------------------ unit kernels */
/* mathematics/intersection_taichi.py:69-91 (e1, e2 computed from f32 vertices) */
static inline int mt_hit(v3 v0, v3 e1, v3 e2, v3 ro, v3 rd, float t0, float t1, float* tout) {
    float t = 3.402823466e+38f; /* MAX_F */
    int hit = 0;
    v3 c = cross(e1, rd);
    float det = dot(c, e2);
    if (fabsf(det) > 0.0f) {
        float f = 1.0f / det;
        v3 s = sub(ro, v0);
        v3 q = cross(s, e2);
        float dse = dot(q, e1);
        t = -f * dse;
        if (t0 < t && t < t1) {
            float u = -f * dot(q, rd);
            if (0.0f <= u && u <= 1.0f) {
                float v = f * dot(c, s);
                if (v >= 0.0f && 1.0f - u - v >= 0.0f) hit = 1;
            }
        }
    }
    *tout = t;
    return hit;
}

/* accelerators/bvh_taichi.py:168-190; factor = f32(1 + 2*GAMMA2_3) */
static float g_gamma_factor = 0x1.000006p+0f; /* 1 + 3*2^-23 */
static inline int aabb_hit(const float* lo, const float* hi, v3 ro, v3 rd, float t0, float t1) {
    int intersect = 1;
    const float o[3] = {ro.x, ro.y, ro.z}, d[3] = {rd.x, rd.y, rd.z};
    for (int i = 0; i < 3; ++i) {
        float tn = (lo[i] - o[i]) / d[i];
        float tf = (hi[i] - o[i]) / d[i];
        if (tn > tf) { float tmp = tn; tn = tf; tf = tmp; }
        tf *= g_gamma_factor;
        if (tn > t0) t0 = tn;
        if (tf < t1) t1 = tf;
        if (t0 > t1) intersect = 0;
    }
    return intersect;
}

/* Trig mode 0 (the spec shared with the HIP kernel): minimax polynomials.
 * Trig mode 1 (reference replay only): theta exactly as samplers.py:16/19
 * computes it, then correctly rounded cos/sin — what the fixture generator's
 * stand-in uses, so scripted replays isolate estimator semantics from trig ulps. */
static int g_trig_mode = 0;
static const float kPiOver2 = 1.57079632679489661923f;

/* mathematics/samplers.py:9-25 */
static inline void concentric_disk(float u0, float u1, float* dx, float* dy) {
    float ox = 2.0f * u0 - 1.0f, oy = 2.0f * u1 - 1.0f;
    if (ox == 0.0f && oy == 0.0f) { *dx = 0.0f; *dy = 0.0f; return; }
    float r, c, s;
    if (fabsf(ox) > fabsf(oy)) {
        r = ox;
        float th = kPiOver4 * (oy / ox);
        if (g_trig_mode) { c = (float)cos((double)th); s = (float)sin((double)th); }
        else { c = poly_cos(th); s = poly_sin(th); }
    } else {
        r = oy;
        float a = kPiOver4 * (ox / oy);  /* theta = pi/2 - a */
        if (g_trig_mode) {
            float th = kPiOver2 - a;
            c = (float)cos((double)th); s = (float)sin((double)th);
        } else { c = poly_sin(a); s = poly_cos(a); }
    }
    *dx = r * c; *dy = r * s;
}

/* mathematics/samplers.py:28-32 */
static inline v3 cosine_hemisphere(float u0, float u1) {
    float dx, dy;
    concentric_disk(u0, u1, &dx, &dy);
    float m = 1.0f - dx * dx - dy * dy;
    float z = sqrtf(m > 0.0f ? m : 0.0f);
    return mk(dx, dy, z);
}

/* mathematics/mat4_taichi.py:9-52 — rows (x, z, n) of rotate_z_to */
static inline void frame_rows(v3 n, v3* r1, v3* r2, v3* r3) {
    v3 v = normalize(n);
    if (v.y == 1.0f) {            /* abs(v.y - 1) < EPS(f32 tiny) */
        *r1 = mk(1, 0, 0); *r2 = mk(0, 0, 1); *r3 = mk(0, 1, 0);
    } else if (v.y == -1.0f) {
        *r1 = mk(1, 0, 0); *r2 = mk(0, 0, 1); *r3 = mk(0, -1, 0);
    } else {
        v3 x = normalize(cross(v, mk(0.0f, 1.0f, 0.0f)));
        v3 z = normalize(cross(x, v));
        *r1 = x; *r2 = z; *r3 = v;
    }
}

/* mathematics/mat4_taichi.py:55-60 */
static inline v3 rotate_vector(v3 r1, v3 r2, v3 r3, v3 a) {
    v3 o = add(add(scl(r1, a.x), scl(r2, a.y)), scl(r3, a.z));
    return normalize(o);
}

/* core/camera_taichi.py:47-74. cam[0..15] = iview columns c1..c4 (rows of
 * iview.T), cam[16..19] = sensor_dim (sw, sh, focus, aperture). */
static inline void gen_ray(const float* cam, float u, float v, Rng* rng, v3* o, v3* d) {
    const float* c1 = cam; const float* c2 = cam + 4; const float* c3 = cam + 8; const float* c4 = cam + 12;
    const float* sd = cam + 16;
    float rdir[4] = {(u - 0.5f) * sd[0] / 0.5f, (v - 0.5f) * sd[1] / 0.5f, -sd[2], 1.0f};
    float rorg[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    if (sd[3] > 0.0f) {  /* quirk kept: jitter scaled by focus distance */
        rorg[0] = sd[2] * rng_next(rng) - sd[2] / 2.0f;
        rorg[1] = sd[2] * rng_next(rng) - sd[2] / 2.0f;
    }
    float dw[4], ow[4];
    const float* cols[4] = {c1, c2, c3, c4};
    for (int i = 0; i < 4; ++i) {
        const float* c = cols[i];
        dw[i] = rdir[0] * c[0] + rdir[1] * c[1] + rdir[2] * c[2] + rdir[3] * c[3];
        ow[i] = rorg[0] * c[0] + rorg[1] * c[1] + rorg[2] * c[2] + rorg[3] * c[3];
    }
    float f[4] = {dw[0] - ow[0], dw[1] - ow[1], dw[2] - ow[2], dw[3] - ow[3]};
    float l = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2] + f[3] * f[3]);
    *o = mk(ow[0], ow[1], ow[2]);
    *d = mk(f[0] / l, f[1] / l, f[2] / l);
}

/* mathematics/intersection_taichi.py:15-36 */
static inline int sphere_hit(v3 c, float radius, v3 ro, v3 rd, float t_min, float t_max, float* root_out) {
    v3 oc = sub(ro, c);
    float a = dot(rd, rd);
    float half_b = dot(oc, rd);
    float cc = dot(oc, oc) - radius * radius;
    float disc = half_b * half_b - a * cc;
    int hit = disc >= 0.0f;
    float root = -1.0f;
    if (hit) {
        float sq = sqrtf(disc);
        root = (-half_b - sq) / a;
        if (root < t_min || t_max < root) {
            root = (-half_b + sq) / a;
            if (root < t_min || t_max < root) hit = 0;
        }
    }
    *root_out = root;
    return hit;
}

/* core/bsdf_taichi.py:6-22 */
static inline float schlick(float cosine, float idx) {
    float r0 = (1.0f - idx) / (1.0f + idx);
    r0 = r0 * r0;
    float m = 1.0f - cosine;
    return r0 + (1.0f - r0) * (m * m * m * m * m);
}
static inline v3 reflect3(v3 v, v3 n) { return sub(v, scl(n, 2.0f * dot(v, n))); }
static inline v3 refract3(v3 v, v3 n, float eta) {
    float ct = -dot(v, n);
    if (ct > 1.0f) ct = 1.0f;
    v3 perp = scl(add(v, scl(n, ct)), eta);
    float k = 1.0f - dot(perp, perp);
    v3 par = scl(n, -sqrtf(fabsf(k)));
    return add(perp, par);
}

/* random_in_unit_sphere (vec3_taichi.py:299-306): theta = 2 pi u1,
 * cos(phi) = 2 u2 - 1, r = u3^(1/3).  Restated with deterministic f32 ops
 * (quadrant reduction + the minimax polynomials, Newton cube root) so CPU
 * and GPU draw identical points; acos is not needed (sin(phi) = sqrt(1-z^2)). */
static inline float cbrt_spec(float x) {
    if (!(x > 0.0f)) return 0.0f;
    union { float f; uint32_t u; } b;
    b.f = x;
    b.u = b.u / 3u + 709921077u;
    float y = b.f;
    for (int i = 0; i < 3; ++i) y = (2.0f * y + x / (y * y)) / 3.0f;
    return y;
}
static inline void sincos_2pi(float u, float* c, float* sn) {
    int q = (int)floorf(u * 4.0f + 0.5f);
    float a = 6.28318530717958647692f * (u - 0.25f * (float)q);   /* in [-pi/4, pi/4] */
    float pc = poly_cos(a), ps = poly_sin(a);
    switch (q & 3) {
        case 0: *c = pc; *sn = ps; break;
        case 1: *c = -ps; *sn = pc; break;
        case 2: *c = -pc; *sn = -ps; break;
        default: *c = ps; *sn = -pc; break;
    }
}
static inline v3 random_in_unit_sphere(Rng* rng) {
    float u1 = rng_next(rng), u2 = rng_next(rng), u3 = rng_next(rng);
    float c, sn;
    sincos_2pi(u1, &c, &sn);
    float z = 2.0f * u2 - 1.0f;
    float m = 1.0f - z * z;
    float sp = sqrtf(m > 0.0f ? m : 0.0f);
    float r = cbrt_spec(u3);
    return mk(r * sp * c, r * sp * sn, r * z);
}

/* ------------------------------------------------------------------ scene */
typedef struct {
    /* triangles (original order) */
    int64_t n_tri;
    float* v0; float* e1; float* e2;   /* n_tri x 3 each */
    float* vtx;                        /* n_tri x 9 original vertices */
    float* nrm;                        /* n_tri x 3 */
    int32_t* mat_id;                   /* n_tri */
    int32_t* prim_id;                  /* n_tri */
    /* materials: rho.rgb, emit, sided, type, ior, roughness */
    int32_t n_mat;
    float* mat;
    /* spheres (build-added primitive; hit = intersection_taichi.py:15-36) */
    int64_t n_sph;
    float* sph;                        /* n_sph x 4: center, radius */
    int32_t* sph_mat;
    /* lights */
    int32_t n_light;
    int32_t* light_tri;
    int32_t* light_off;
    float direct_rgb[3];
    /* optional external BVH2 (prt_bvh_export layout) for the BACKEND_BVH traversal */
    int64_t x_nodes;
    float* xnode;                      /* x_nodes x 16 */
    int32_t* xorder;                   /* BVH slot -> triangle */
    /* reference-structure BVH over primitives (bvh_taichi.py) */
    int32_t n_prim;
    int32_t* prim_first; int32_t* prim_count;
    int32_t n_node;
    int32_t* bobj; int32_t* bleft; int32_t* bright; int32_t* bnext;
    float* bmin; float* bmax;
} OScene;

typedef struct { int32_t lo, hi; int32_t id; int32_t parent; int32_t left, right; float mn[3], mx[3]; } BNode;

static int build_ref_node(BNode* nodes, int* count, const float* plo, const float* phi,
                          int lo, int hi, int parent) {
    int me = (*count)++;
    BNode* n = &nodes[me];
    n->lo = lo; n->hi = hi; n->parent = parent; n->left = n->right = -1;
    int span = hi - lo;
    if (span == 1) {
        for (int k = 0; k < 3; ++k) { n->mn[k] = plo[3 * lo + k]; n->mx[k] = phi[3 * lo + k]; }
    } else {
        int mid = lo + span / 2;  /* accelerators/bvh_taichi.py:79-81 */
        int l = build_ref_node(nodes, count, plo, phi, lo, mid, me);
        int r = build_ref_node(nodes, count, plo, phi, mid, hi, me);
        n = &nodes[me];
        n->left = l; n->right = r;
        for (int k = 0; k < 3; ++k) {
            n->mn[k] = fminf(nodes[l].mn[k], nodes[r].mn[k]);
            n->mx[k] = fmaxf(nodes[l].mx[k], nodes[r].mx[k]);
        }
    }
    return me;
}

OR_API void or_set_gamma_factor(float g) { g_gamma_factor = g; }
OR_API void or_set_trig_mode(int m) { g_trig_mode = m; }

OR_API void* or_scene_create(const float* tri_v, const float* tri_n, const int32_t* tri_mat,
                             const int32_t* tri_prim, int64_t n_tri,
                             const float* prim_lo, const float* prim_hi, int32_t n_prim,
                             const float* sph, const int32_t* sph_mat, int64_t n_sph,
                             const float* mat, int32_t n_mat,
                             const int32_t* light_tri, const int32_t* light_off, int32_t n_light,
                             const float* direct_rgb) {
    OScene* s = (OScene*)calloc(1, sizeof(OScene));
    s->n_sph = n_sph;
    s->sph = (float*)malloc(sizeof(float) * 4 * (n_sph > 0 ? n_sph : 1));
    s->sph_mat = (int32_t*)malloc(sizeof(int32_t) * (n_sph > 0 ? n_sph : 1));
    if (n_sph > 0) {
        memcpy(s->sph, sph, sizeof(float) * 4 * n_sph);
        memcpy(s->sph_mat, sph_mat, sizeof(int32_t) * n_sph);
    }
    s->n_tri = n_tri;
    s->v0 = (float*)malloc(sizeof(float) * 3 * n_tri);
    s->e1 = (float*)malloc(sizeof(float) * 3 * n_tri);
    s->e2 = (float*)malloc(sizeof(float) * 3 * n_tri);
    s->vtx = (float*)malloc(sizeof(float) * 9 * n_tri);
    s->nrm = (float*)malloc(sizeof(float) * 3 * n_tri);
    s->mat_id = (int32_t*)malloc(sizeof(int32_t) * n_tri);
    s->prim_id = (int32_t*)malloc(sizeof(int32_t) * n_tri);
    memcpy(s->vtx, tri_v, sizeof(float) * 9 * n_tri);
    memcpy(s->nrm, tri_n, sizeof(float) * 3 * n_tri);
    memcpy(s->mat_id, tri_mat, sizeof(int32_t) * n_tri);
    for (int64_t i = 0; i < n_tri; ++i) {
        const float* t = tri_v + 9 * i;
        for (int k = 0; k < 3; ++k) {
            s->v0[3 * i + k] = t[k];
            s->e1[3 * i + k] = t[3 + k] - t[k];
            s->e2[3 * i + k] = t[6 + k] - t[k];
        }
        s->prim_id[i] = tri_prim ? tri_prim[i] : 0;
    }
    s->n_mat = n_mat;
    s->mat = (float*)malloc(sizeof(float) * 8 * n_mat);
    memcpy(s->mat, mat, sizeof(float) * 8 * n_mat);
    s->n_light = n_light;
    s->light_off = (int32_t*)malloc(sizeof(int32_t) * (n_light + 1));
    memcpy(s->light_off, light_off, sizeof(int32_t) * (n_light + 1));
    s->light_tri = (int32_t*)malloc(sizeof(int32_t) * (light_off[n_light] > 0 ? light_off[n_light] : 1));
    memcpy(s->light_tri, light_tri, sizeof(int32_t) * light_off[n_light]);
    memcpy(s->direct_rgb, direct_rgb, sizeof(float) * 3);
    /* reference-structure BVH over primitives (insertion order, median split) */
    if (tri_prim && n_prim > 0) {
        s->n_prim = n_prim;
        s->prim_first = (int32_t*)calloc(n_prim, sizeof(int32_t));
        s->prim_count = (int32_t*)calloc(n_prim, sizeof(int32_t));
        for (int p = 0; p < n_prim; ++p) s->prim_first[p] = -1;
        for (int64_t i = 0; i < n_tri; ++i) {
            int p = tri_prim[i];
            if (s->prim_first[p] < 0) s->prim_first[p] = (int32_t)i;
            s->prim_count[p]++;
        }
        BNode* nodes = (BNode*)calloc(2 * n_prim, sizeof(BNode));
        int count = 0;
        build_ref_node(nodes, &count, prim_lo, prim_hi, 0, n_prim, -1);
        /* preorder ids == creation order here (left subtree built before right) */
        s->n_node = count;
        s->bobj = (int32_t*)malloc(sizeof(int32_t) * count);
        s->bleft = (int32_t*)malloc(sizeof(int32_t) * count);
        s->bright = (int32_t*)malloc(sizeof(int32_t) * count);
        s->bnext = (int32_t*)malloc(sizeof(int32_t) * count);
        s->bmin = (float*)malloc(sizeof(float) * 3 * count);
        s->bmax = (float*)malloc(sizeof(float) * 3 * count);
        for (int i = 0; i < count; ++i) {
            BNode* n = &nodes[i];
            s->bobj[i] = (n->left < 0 && n->right < 0) ? n->lo : -1;
            s->bleft[i] = n->left;
            s->bright[i] = n->right;
            /* BVHNode.next (bvh_taichi.py:92-104) */
            int cur = i, nx = -1;
            while (1) {
                int par = nodes[cur].parent;
                if (par >= 0 && nodes[par].right != cur) { nx = nodes[par].right; break; }
                if (par < 0) { nx = -1; break; }
                cur = par;
            }
            s->bnext[i] = nx;
            for (int k = 0; k < 3; ++k) { s->bmin[3 * i + k] = n->mn[k]; s->bmax[3 * i + k] = n->mx[k]; }
        }
        free(nodes);
    }
    return s;
}

OR_API void or_scene_destroy(void* p) {
    OScene* s = (OScene*)p;
    if (!s) return;
    free(s->v0); free(s->e1); free(s->e2); free(s->vtx); free(s->nrm); free(s->mat_id); free(s->prim_id);
    free(s->mat); free(s->light_tri); free(s->light_off); free(s->sph); free(s->sph_mat);
    free(s->xnode); free(s->xorder);
    free(s->prim_first); free(s->prim_count);
    free(s->bobj); free(s->bleft); free(s->bright); free(s->bnext); free(s->bmin); free(s->bmax);
    free(s);
}

OR_API int or_ref_bvh(void* p, int32_t* obj, int32_t* left, int32_t* right, int32_t* next, float* mn, float* mx) {
    OScene* s = (OScene*)p;
    for (int i = 0; i < s->n_node; ++i) {
        obj[i] = s->bobj[i]; left[i] = s->bleft[i]; right[i] = s->bright[i]; next[i] = s->bnext[i];
        for (int k = 0; k < 3; ++k) { mn[3 * i + k] = s->bmin[3 * i + k]; mx[3 * i + k] = s->bmax[3 * i + k]; }
    }
    return s->n_node;
}

static inline v3 tri_v0(const OScene* s, int64_t i) { return ld3(s->v0 + 3 * i); }
static inline v3 tri_e1(const OScene* s, int64_t i) { return ld3(s->e1 + 3 * i); }
static inline v3 tri_e2(const OScene* s, int64_t i) { return ld3(s->e2 + 3 * i); }
static inline const float* matp(const OScene* s, int64_t tri) { return s->mat + 8 * s->mat_id[tri]; }

/* Hit id space: [0, n_tri) triangles, [n_tri, n_tri + n_sph) spheres. */
static inline const float* mat_of(const OScene* s, int64_t id) {
    if (id < s->n_tri) return s->mat + 8 * s->mat_id[id];
    return s->mat + 8 * s->sph_mat[id - s->n_tri];
}
/* geometric (unflipped) normal: stored face normal, or (p - c) / r for spheres */
static inline v3 geo_normal(const OScene* s, int64_t id, v3 p) {
    if (id < s->n_tri) return ld3(s->nrm + 3 * id);
    const float* c = s->sph + 4 * (id - s->n_tri);
    return mk((p.x - c[0]) / c[3], (p.y - c[1]) / c[3], (p.z - c[2]) / c[3]);
}

/* Shading frame + scatter of Quad.hit/Cube.hit (shapes.py:98-108): flip the
 * face normal toward the ray for two-sided BSDFs, draw the cosine-hemisphere
 * direction, rotate it into the normal frame, pdf = |n.wi|/pi. */
static inline v3 shade_normal(const OScene* s, int64_t tri, v3 rd) {
    v3 n = ld3(s->nrm + 3 * tri);
    const float* m = matp(s, tri);
    if (m[4] == 0.0f && dot(n, neg(rd)) < 0.0f) n = neg(n);
    return n;
}
static inline void scatter(Rng* rng, v3 n, v3* wi, float* pdf) {
    float u0 = rng_next(rng);
    float u1 = rng_next(rng);
    v3 l = cosine_hemisphere(u0, u1);
    v3 r1, r2, r3;
    frame_rows(n, &r1, &r2, &r3);
    *wi = rotate_vector(r1, r2, r3, l);
    *pdf = fabsf(dot(n, *wi)) * kInvPi;
}

typedef struct { int hit; float t; int64_t tri; v3 n; v3 wi; float pdf; } Hit;

/* World.hit_all over the reference-structure BVH (intersection_taichi.py:238-291).
 * draws != 0 replays the reference's RNG consumption: every primitive that
 * improves the closest hit draws its scatter direction (shapes.py:105). */
static Hit hit_all_ref(const OScene* s, v3 ro, v3 rd, float t_min, float closest, Rng* rng, int draws,
                       uint64_t* cnt) {
    Hit h; memset(&h, 0, sizeof(h));
    int curr = 0;
    while (curr != -1) {
        int obj = s->bobj[curr];
        if (obj != -1) {
            /* Quad.hit / Cube.hit: loop faces, shrink t1 */
            float t1 = closest, tbest = 3.402823466e+38f;
            int any = 0; int64_t face = 0;
            int64_t f0 = s->prim_first[obj], fc = s->prim_count[obj];
            for (int64_t i = f0; i < f0 + fc; ++i) {
                float t;
                if (cnt) cnt[1]++;
                int hh = mt_hit(tri_v0(s, i), tri_e1(s, i), tri_e2(s, i), ro, rd, t_min, t1, &t);
                if (hh && t < tbest) { t1 = t; tbest = t; face = i; any = 1; }
            }
            if (any) {
                v3 n = shade_normal(s, face, rd);
                v3 wi = mk(0, 0, 0); float pdf = 0.0f;
                if (draws) scatter(rng, n, &wi, &pdf);
                h.hit = 1; closest = tbest; h.tri = face; h.n = n; h.wi = wi; h.pdf = pdf;
            }
            curr = s->bnext[curr];
        } else {
            if (cnt) cnt[0]++;
            if (aabb_hit(s->bmin + 3 * curr, s->bmax + 3 * curr, ro, rd, t_min, closest)) {
                if (s->bleft[curr] != -1) curr = s->bleft[curr];
                else if (s->bright[curr] != -1) curr = s->bright[curr];
                else curr = s->bnext[curr];
            } else {
                curr = s->bnext[curr];
            }
        }
    }
    h.t = closest;
    return h;
}

/* Brute force over all triangles: closest (t, index), strict t0 < t < t1. */
static Hit hit_all_brute(const OScene* s, v3 ro, v3 rd, float t_min, float t_max, int any_hit, uint64_t* cnt) {
    Hit h; memset(&h, 0, sizeof(h));
    float best = t_max;
    for (int64_t i = 0; i < s->n_tri; ++i) {
        float t;
        if (mt_hit(tri_v0(s, i), tri_e1(s, i), tri_e2(s, i), ro, rd, t_min, best, &t)) {
            best = t; h.hit = 1; h.tri = i;
            if (any_hit) break;
        }
    }
    if (cnt) cnt[1] += (uint64_t)s->n_tri;
    if (!(any_hit && h.hit)) {
        for (int64_t k = 0; k < s->n_sph; ++k) {
            float root;
            const float* c = s->sph + 4 * k;
            if (sphere_hit(mk(c[0], c[1], c[2]), c[3], ro, rd, t_min, best, &root)) {
                best = root; h.hit = 1; h.tri = s->n_tri + k;
                if (any_hit) break;
            }
        }
    }
    h.t = best;
    return h;
}

/* Traversal of an external BVH2 (nodes from prt_bvh_export: two child boxes +
 * refs per 64-B node; leaf ref < 0 encodes (first slot, count)).  Boxes only
 * prune, so the result is the brute-force closest (t, index) hit; the slab test
 * is the reference's (bvh_taichi.py:168-190) with t1 = closest so far. */
static Hit hit_all_bvh(const OScene* s, v3 ro, v3 rd, float t_min, float t_max, int any_hit, uint64_t* cnt) {
    Hit h; memset(&h, 0, sizeof(h));
    float best = t_max;
    int64_t best_id = -1;
    int32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        int32_t cur = stack[--sp];
        if (cur >= 0) {
            const float* nd = s->xnode + 16 * (int64_t)cur;
            if (cnt) cnt[0]++;
            for (int side = 1; side >= 0; --side) {
                const float* b = nd + 6 * side;
                float lo[3] = {b[0], b[2], b[4]}, hi[3] = {b[1], b[3], b[5]};
                if (aabb_hit(lo, hi, ro, rd, t_min, best)) {
                    int32_t ref;
                    memcpy(&ref, nd + 12 + side, 4);
                    if (sp < 128) stack[sp++] = ref;
                }
            }
        } else {
            int32_t v = -cur - 1;
            int64_t first = v >> 3, count = (v & 7) + 1;
            for (int64_t k = first; k < first + count; ++k) {
                int64_t i = s->xorder[k];
                float t;
                if (cnt) cnt[1]++;
                if (mt_hit(tri_v0(s, i), tri_e1(s, i), tri_e2(s, i), ro, rd, t_min, t_max, &t) &&
                    (t < best || (t == best && best_id >= 0 && i < best_id))) {
                    best = t; best_id = i;
                    if (any_hit) { sp = 0; break; }
                }
            }
        }
    }
    h.hit = best_id >= 0;
    h.tri = best_id;
    if (!(any_hit && h.hit)) {
        for (int64_t k = 0; k < s->n_sph; ++k) {
            float root;
            const float* c = s->sph + 4 * k;
            if (sphere_hit(mk(c[0], c[1], c[2]), c[3], ro, rd, t_min, best, &root)) {
                best = root; h.hit = 1; h.tri = s->n_tri + k;
                if (any_hit) break;
            }
        }
    }
    h.t = best;
    return h;
}

/* order: BVH slot -> triangle, n_order entries (>= n_tri: the build may reference a large
 * triangle from several leaves, early split clipping; each slot is tested like a leaf entry) */
OR_API int or_scene_set_bvh(void* p, const float* nodes, int64_t n_nodes, const int32_t* order, int64_t n_order) {
    OScene* s = (OScene*)p;
    free(s->xnode); free(s->xorder);
    s->x_nodes = n_nodes;
    s->xnode = (float*)malloc(sizeof(float) * 16 * n_nodes);
    s->xorder = (int32_t*)malloc(sizeof(int32_t) * (n_order > 0 ? n_order : 1));
    memcpy(s->xnode, nodes, sizeof(float) * 16 * n_nodes);
    memcpy(s->xorder, order, sizeof(int32_t) * n_order);
    return 0;
}

enum { BACKEND_REF = 0, BACKEND_BRUTE = 1, BACKEND_BVH = 2 };

static Hit closest_hit(const OScene* s, int backend, v3 ro, v3 rd, float t0, float t1, uint64_t* cnt) {
    if (backend == BACKEND_REF) return hit_all_ref(s, ro, rd, t0, t1, NULL, 0, cnt);
    Hit h = backend == BACKEND_BVH ? hit_all_bvh(s, ro, rd, t0, t1, 0, cnt) : hit_all_brute(s, ro, rd, t0, t1, 0, cnt);
    if (h.hit) {
        v3 ng = geo_normal(s, h.tri, add(ro, scl(rd, h.t)));
        const float* m = mat_of(s, h.tri);
        h.n = (m[4] == 0.0f && dot(ng, neg(rd)) < 0.0f) ? neg(ng) : ng;
    }
    return h;
}

static int occluded(const OScene* s, int backend, v3 ro, v3 rd, float t0, float t1, uint64_t* cnt) {
    if (backend == BACKEND_REF) return hit_all_ref(s, ro, rd, t0, t1, NULL, 0, cnt).hit;
    if (backend == BACKEND_BVH) return hit_all_bvh(s, ro, rd, t0, t1, 1, cnt).hit;
    return hit_all_brute(s, ro, rd, t0, t1, 1, cnt).hit;
}

/* World.sample_a_light + Quad.sample_a_point (intersection_taichi.py:194-207,
 * shapes.py:62-71) */
static inline void sample_light(const OScene* s, Rng* rng, v3* p2, v3* n2, v3* e) {
    int li = 0;
    if (s->n_light > 1) li = rng_int(rng, 0, s->n_light - 1);
    int nf = s->light_off[li + 1] - s->light_off[li];
    int f = rng_int(rng, 0, nf - 1);
    int64_t tri = s->light_tri[s->light_off[li] + f];
    float u = sqrtf(rng_next(rng));
    float v = rng_next(rng);
    float a = u * (1.0f - v);
    float b = u * v;
    const float* t = s->vtx + 9 * tri;
    v3 V0 = ld3(t), V1 = ld3(t + 3), V2 = ld3(t + 6);
    float c = 1.0f - a - b;
    *p2 = add(add(scl(V0, a), scl(V1, b)), scl(V2, c));
    *n2 = ld3(s->nrm + 3 * tri);
    const float* m = matp(s, tri);
    *e = mk(m[0], m[1], m[2]);  /* BSDFLight.evaluate() = (rho, rho, rho) */
}

/* ------------------------------------------- MIS direct lighting (variant) */
/* The reference's unused helpers (core/tracing.py:12-39) and sample_direct_lighting2
 * (core/tracing.py:57-90): one light-sampling and one BRDF-sampling strategy combined
 * with the power heuristic, both visibility tests closest-hit queries over (1e-5,
 * 9999.9) that must land on an emitter, light_area fixed at 1.0 (as the reference
 * passes it), and the BRDF strategy's light pdf taken with the normal n2 of the
 * LIGHT-SAMPLED point (the reference's quirk, kept).  trace() calls it instead of
 * sample_direct_lighting when g_nee_mis is set (or_set_nee_mode). */
static int g_nee_mis = 0;
static const float kPiF = 3.14159265358979323846f;   /* np.pi in a Taichi f32 kernel */
static const float kTMaxMis = 9999.9f;                /* core/tracing.py:67,80 */

static inline float dot_or_zero(v3 n, v3 l) { float d = dot(n, l); return 0.0f > d ? 0.0f : d; }
static inline float mis_power(float pf, float pg) {
    float f = pf * pf, g = pg * pg;
    return f / (f + g);
}
static inline float area_light_pdf(float t_light, v3 dir, v3 light_n, float light_area) {
    float pdf = 0.0f;
    float l_cos = dot(light_n, neg(dir));
    if (l_cos > 1e-4f) {
        v3 tmp = scl(dir, t_light);
        float dist_sqr = dot(tmp, tmp);
        pdf = dist_sqr / (light_area * l_cos);
    }
    return pdf;
}
static inline float brdf_pdf_of(v3 n, v3 dir) { return dot_or_zero(n, dir) / kPiF; }

/* closest hit for the MIS queries; *emit = emitting_light of the hit primitive */
static Hit mis_query(const OScene* s, int backend, v3 o, v3 d, Rng* rng, int scripted, uint64_t* cnt) {
    if (cnt) cnt[3]++;
    if (scripted) return hit_all_ref(s, o, d, kTMin, kTMaxMis, rng, 1, cnt);
    return closest_hit(s, backend, o, d, kTMin, kTMaxMis, cnt);
}

static v3 direct_mis(const OScene* s, int backend, v3 p, v3 n, v3 rho, Rng* rng, int scripted, uint64_t* cnt) {
    v3 p2, n2, e;
    sample_light(s, rng, &p2, &n2, &e);
    v3 direct = mk(0, 0, 0);
    v3 fl = mul(scl(rho, kInvPi), e);   /* InvPi * hit_color * light_color */
    v3 tl = normalize(sub(p2, p));
    if (dot(tl, n) > 0.0f) {
        Hit h = mis_query(s, backend, p, tl, rng, scripted, cnt);
        if (h.hit && mat_of(s, h.tri)[3] > 0.0f) {
            float lp = area_light_pdf(h.t, tl, n2, 1.0f);
            float bp = brdf_pdf_of(n, tl);
            if (lp > 0.0f && bp > 0.0f) {
                float w = mis_power(lp, bp);
                float nl = dot_or_zero(tl, n);
                direct = add(direct, mk(fl.x * w * nl / lp, fl.y * w * nl / lp, fl.z * w * nl / lp));
            }
        }
    }
    v3 bd; float bp;
    scatter(rng, n, &bd, &bp);   /* cosine_sample_hemisphere_convenient(hit_normal) */
    if (bp > 0.0f) {
        Hit h = mis_query(s, backend, p, bd, rng, scripted, cnt);
        if (h.hit && mat_of(s, h.tri)[3] > 0.0f) {
            float lp = area_light_pdf(h.t, bd, n2, 1.0f);
            if (lp > 0.0f) {
                float w = mis_power(bp, lp);
                float nl = dot_or_zero(bd, n);
                direct = add(direct, mk(fl.x * w * nl / bp, fl.y * w * nl / bp, fl.z * w * nl / bp));
            }
        }
    }
    return direct;
}

/* PathTracer.trace (core/tracing.py:116-155): the radiance of one path from (ro, rd). */
static v3 trace_path(const OScene* s, int backend, v3 ro, v3 rd, int depth, Rng* rng, int scripted, uint64_t* cnt) {
    v3 L = mk(0, 0, 0), beta = mk(1, 1, 1);
    v3 lc = mk(s->direct_rgb[0], s->direct_rgb[1], s->direct_rgb[2]);
    for (int b = 0; b < depth; ++b) {
        Hit h;
        if (cnt) cnt[2]++;
        if (scripted) h = hit_all_ref(s, ro, rd, kTMin, kTMax, rng, 1, cnt);
        else h = closest_hit(s, backend, ro, rd, kTMin, kTMax, cnt);
        if (!h.hit) break;
        const float* m = mat_of(s, h.tri);
        v3 n = h.n;
        if (m[3] != 0.0f) {  /* emitter: tracing.py:129-139 */
            float d1 = dot(neg(rd), n);
            if (d1 > 0.0f) {
                if (b == 0) L = add(L, mul(lc, beta));
                else L = add(L, scl(mul(lc, beta), d1));
            }
            break;
        }
        if (m[5] == 2.0f || m[5] == 3.0f) {
            /* specular BSDFs (build-added, config 3): bsdf_taichi.py:52-59 / :69-86.
             * Delta distributions: beta *= albedo, no NEE, next ray = the scattered one. */
            v3 p = add(ro, scl(rd, h.t));
            v3 ng = geo_normal(s, h.tri, p);
            int front = dot(rd, ng) < 0.0f;
            v3 ns = front ? ng : neg(ng);
            v3 unit = normalize(rd);
            v3 out;
            if (m[5] == 2.0f) {
                out = reflect3(unit, ns);
                if (m[7] > 0.0f) out = add(out, scl(random_in_unit_sphere(rng), m[7]));
                if (!(dot(out, ns) > 0.0f)) break;   /* absorbed */
            } else {
                float ratio = front ? 1.0f / m[6] : m[6];
                float ct = -dot(unit, ns);
                if (ct > 1.0f) ct = 1.0f;
                float st = sqrtf(1.0f - ct * ct);
                int cannot = ratio * st > 1.0f;
                if (cannot || schlick(ct, ratio) > rng_next(rng)) out = reflect3(unit, ns);
                else out = refract3(unit, ns, ratio);
            }
            beta = mul(beta, mk(m[0], m[1], m[2]));
            ro = p; rd = normalize(out);
            continue;
        }
        v3 wi; float pdf;
        if (scripted) { wi = h.wi; pdf = h.pdf; }
        else scatter(rng, n, &wi, &pdf);
        v3 p = add(ro, scl(rd, h.t));   /* ray.at: o + d*t */
        v3 att = mk(m[0], m[1], m[2]);
        float cw = dot(n, wi);
        float dz = cw > 0.0f ? cw : 0.0f;  /* dot_or_zero = max(0, n.wi) */
        v3 nb = mk(att.x * dz / pdf * kInvPi, att.y * dz / pdf * kInvPi, att.z * dz / pdf * kInvPi);
        if (isnan(nb.x) || isnan(nb.y) || isnan(nb.z)) {
            pdf = 1e-4f;
            nb = mk(att.x * dz / pdf * kInvPi, att.y * dz / pdf * kInvPi, att.z * dz / pdf * kInvPi);
        }
        beta = mul(beta, nb);
        if (g_nee_mis) {
            /* variant: L += beta * sample_direct_lighting2(hit_pos, normal, attenuation) */
            L = add(L, mul(beta, direct_mis(s, backend, p, n, att, rng, scripted, cnt)));
            ro = p; rd = wi;
            continue;
        }
        /* sample_direct_lighting (tracing.py:92-108) */
        v3 p2, n2, e;
        sample_light(s, rng, &p2, &n2, &e);
        v3 w = normalize(sub(p2, p));
        v3 w2 = normalize(sub(p, p2));
        float t_at = (p2.x - p.x) / w.x;
        int blocked;
        if (scripted) {
            if (cnt) cnt[3]++;
            blocked = hit_all_ref(s, p, w, kTMin, t_at, rng, 1, cnt).hit;
        } else {
            /* the shadow query is only issued when it can contribute */
            float dot1 = dot(n, w), dot2 = dot(n2, w2);
            if (dot1 > 0.0f && dot2 > 0.0f) {
                if (cnt) cnt[3]++;
                blocked = occluded(s, backend, p, w, kTMin, t_at, cnt);
            } else {
                blocked = 1;
            }
        }
        if (!blocked) {
            float dot1 = dot(n, w), dot2 = dot(n2, w2);
            if (dot1 > 0.0f && dot2 > 0.0f) {
                v3 d = sub(p, p2);
                float sl = dot(d, d);
                v3 rad = mk(e.x * dot1 * dot2 / sl, e.y * dot1 * dot2 / sl, e.z * dot1 * dot2 / sl);
                L = add(L, mul(beta, rad));
            }
        }
        ro = p; rd = wi;
    }
    return L;
}

/* render() sample body (main_taichi.py:93-97): camera jitter, gen_ray, trace. */
static v3 trace_sample(const OScene* s, int backend, const float* cam, int W, int H, int x, int y,
                       int depth, Rng* rng, int scripted, uint64_t* cnt) {
    float r0 = rng_next(rng);
    float u = ((float)x + r0) / (float)(W - 1);
    float r1 = rng_next(rng);
    float v = ((float)y + r1) / (float)(H - 1);
    v3 ro, rd;
    gen_ray(cam, u, v, rng, &ro, &rd);
    return trace_path(s, backend, ro, rd, depth, rng, scripted, cnt);
}

/* ------------------------------------------------------------ public API */
OR_API int or_mt(const float* v0, const float* v1, const float* v2, const float* ro, const float* rd,
                 float t0, float t1, float* t) {
    v3 a = ld3(v0), b = ld3(v1), c = ld3(v2);
    return mt_hit(a, sub(b, a), sub(c, a), ld3(ro), ld3(rd), t0, t1, t);
}
OR_API int or_aabb(const float* lo, const float* hi, const float* ro, const float* rd, float t0, float t1) {
    return aabb_hit(lo, hi, ld3(ro), ld3(rd), t0, t1);
}
OR_API void or_disk(const float* u, float* out) { concentric_disk(u[0], u[1], out, out + 1); }
OR_API void or_hemi(const float* u, float* out) { st3(out, cosine_hemisphere(u[0], u[1])); }
OR_API void or_frame(const float* n, float* rows9) {
    v3 r1, r2, r3;
    frame_rows(ld3(n), &r1, &r2, &r3);
    st3(rows9, r1); st3(rows9 + 3, r2); st3(rows9 + 6, r3);
}
OR_API void or_rotate(const float* rows9, const float* v, float* out) {
    st3(out, rotate_vector(ld3(rows9), ld3(rows9 + 3), ld3(rows9 + 6), ld3(v)));
}
OR_API void or_gen_ray(const float* cam, float u, float v, float* o, float* d) {
    Rng r; memset(&r, 0, sizeof(r));
    v3 oo, dd;
    gen_ray(cam, u, v, &r, &oo, &dd);
    st3(o, oo); st3(d, dd);
}
OR_API int or_sphere(const float* c, float r, const float* ro, const float* rd, float t0, float t1, float* root) {
    return sphere_hit(ld3(c), r, ld3(ro), ld3(rd), t0, t1, root);
}
OR_API void or_reflect(const float* v, const float* n, float* out) { st3(out, reflect3(ld3(v), ld3(n))); }
OR_API void or_refract(const float* v, const float* n, float eta, float* out) { st3(out, refract3(ld3(v), ld3(n), eta)); }
OR_API float or_schlick(float c, float idx) { return schlick(c, idx); }
OR_API uint32_t or_rng_key(uint64_t seed, uint32_t pixel, uint32_t sample) { return rng_key(seed, pixel, sample); }
OR_API void or_rng_draws(uint32_t key, int n, float* out) {
    Rng r; memset(&r, 0, sizeof(r)); r.state = key;
    for (int i = 0; i < n; ++i) out[i] = rng_next(&r);
}
OR_API void or_sample_light_scripted(void* p, const float* draws, float* p2, float* n2, float* e) {
    OScene* s = (OScene*)p;
    Rng r; memset(&r, 0, sizeof(r)); r.script = draws; r.script_len = 16;
    v3 a, b, c;
    sample_light(s, &r, &a, &b, &c);
    st3(p2, a); st3(n2, b); st3(e, c);
}

OR_API void or_set_nee_mode(int mis) { g_nee_mis = mis ? 1 : 0; }
OR_API float or_mis_power(float pf, float pg) { return mis_power(pf, pg); }
OR_API float or_area_light_pdf(float t, const float* d, const float* n2) { return area_light_pdf(t, ld3(d), ld3(n2), 1.0f); }
OR_API float or_brdf_pdf(const float* n, const float* d) { return brdf_pdf_of(ld3(n), ld3(d)); }
OR_API float or_dot_or_zero(const float* n, const float* d) { return dot_or_zero(ld3(n), ld3(d)); }
/* sample_direct_lighting2 replayed on a scripted stream (reference order, hit_all's draws
 * included); returns the number of draws consumed (-1 on stream overflow) */
OR_API int or_direct_mis_scripted(void* p, const float* pos, const float* nrm, const float* rho, const float* stream,
                                  int stream_len, float* out) {
    OScene* s = (OScene*)p;
    Rng r; memset(&r, 0, sizeof(r));
    r.script = stream; r.script_len = stream_len;
    st3(out, direct_mis(s, BACKEND_REF, ld3(pos), ld3(nrm), ld3(rho), &r, 1, NULL));
    return r.overflow ? -1 : r.pos;
}

/* batch closest-hit: out_hit[i], out_t[i], out_tri[i], out_n[3i] */
OR_API void or_closest_batch(void* p, int backend, int64_t n, const float* ro, const float* rd,
                             const float* t0, const float* t1, int32_t* out_hit, float* out_t,
                             int64_t* out_tri, float* out_n) {
    OScene* s = (OScene*)p;
    /* independent rays, read-only scene: OpenMP over the batch (the brute-force backend's 1 M-triangle
     * checks of config 4, tests/test_gpu_configs.py) */
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t i = 0; i < n; ++i) {
        Hit h = closest_hit(s, backend, ld3(ro + 3 * i), ld3(rd + 3 * i), t0[i], t1[i], NULL);
        out_hit[i] = h.hit; out_t[i] = h.t; out_tri[i] = h.hit ? h.tri : -1;
        st3(out_n + 3 * i, h.hit ? h.n : mk(0, 0, 0));
    }
}

/* World.hit_all's 8-tuple for a batch of rays (intersection_taichi.py:238-291; libprt's
 * prt_hit_all): out16[i] = hit, t (t1 on a miss), p = o + t d, the shading normal (flipped for
 * two-sided BSDFs, shapes.py:101-102), emit, bsdf.evaluate(), the scattered direction and its pdf
 * (bsdf.py:29-34 + shapes.py:105-108), the scatter's two draws from the stream keyed
 * (seed, i, 0); zeros after t on a miss. */
OR_API void or_hit_all_batch(void* p, int backend, int64_t n, const float* ro, const float* rd, const float* t0,
                             const float* t1, uint64_t seed, float* out16) {
    OScene* s = (OScene*)p;
    for (int64_t i = 0; i < n; ++i) {
        v3 o = ld3(ro + 3 * i), d = ld3(rd + 3 * i);
        Hit h = closest_hit(s, backend, o, d, t0[i], t1[i], NULL);
        float* r = out16 + 16 * i;
        memset(r, 0, 16 * sizeof(float));
        r[1] = h.hit ? h.t : t1[i];
        if (!h.hit) continue;
        const float* m = mat_of(s, h.tri);
        Rng rng; memset(&rng, 0, sizeof(rng));
        rng.state = rng_key(seed, (uint32_t)i, 0u);
        v3 wi; float pdf;
        scatter(&rng, h.n, &wi, &pdf);
        r[0] = 1.0f;
        st3(r + 2, add(o, scl(d, h.t)));
        st3(r + 5, h.n);
        r[8] = m[3] != 0.0f ? 1.0f : 0.0f;
        r[9] = m[0]; r[10] = m[1]; r[11] = m[2];
        st3(r + 12, wi);
        r[15] = pdf;
    }
}

/* PathTracer.trace for caller-given rays (libprt's prt_trace_rays): ray i draws from the stream
 * keyed (seed, i, 0). */
OR_API void or_trace_rays(void* p, int backend, int64_t n, const float* ro, const float* rd, int depth, uint64_t seed,
                          int nthreads, float* out) {
    OScene* s = (OScene*)p;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; ++i) {
        Rng rng; memset(&rng, 0, sizeof(rng));
        rng.state = rng_key(seed, (uint32_t)i, 0u);
        st3(out + 3 * i, trace_path(s, backend, ld3(ro + 3 * i), ld3(rd + 3 * i), depth, &rng, 0, NULL));
    }
}

/* PathTracer.trace with a scripted random stream consumed in the reference's
 * order (REF backend). Returns draws used, or -1 if the stream ran out. */
OR_API int or_trace_scripted(void* p, const float* cam, int W, int H, int x, int y, int depth,
                             const float* stream, int stream_len, float* out) {
    OScene* s = (OScene*)p;
    Rng r; memset(&r, 0, sizeof(r));
    r.script = stream; r.script_len = stream_len;
    v3 L = trace_sample(s, BACKEND_REF, cam, W, H, x, y, depth, &r, 1, NULL);
    st3(out, L);
    return r.overflow ? -1 : r.pos;
}

/* Render a tile set (same contract as prt_render_tiles): out_sum[slot*3+c] =
 * sequential f32 sum over samples 0..spp-1 of the radiance of pixel `slot`.
 * Slot order: tile-major, then ly, then lx (x fastest). Pixels outside the
 * W x H frame are left zero. counters (optional, 4 x u64): AABB tests,
 * triangle tests, closest-hit queries, shadow queries. */
OR_API int or_render_tiles(void* p, int backend, const float* cam, int W, int H, int tw, int th,
                           const int32_t* tile_ids, int n_tiles, int spp, int depth, uint64_t seed,
                           int nthreads, float* out_sum, uint64_t* counters) {
    OScene* s = (OScene*)p;
    int64_t n_slots = (int64_t)n_tiles * tw * th;
    int tiles_x = (W + tw - 1) / tw;
    uint64_t tot[4] = {0, 0, 0, 0};
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        uint64_t loc[4] = {0, 0, 0, 0};
#pragma omp for schedule(dynamic, 16)
        for (int64_t slot = 0; slot < n_slots; ++slot) {
            int64_t tile_k = slot / ((int64_t)tw * th);
            int local = (int)(slot % ((int64_t)tw * th));
            int tid = tile_ids[tile_k];
            int x = (tid % tiles_x) * tw + local % tw;
            int y = (tid / tiles_x) * th + local / tw;
            float acc[3] = {0.0f, 0.0f, 0.0f};
            if (x < W && y < H) {
                uint32_t pix = (uint32_t)y * (uint32_t)W + (uint32_t)x;
                for (int smp = 0; smp < spp; ++smp) {
                    Rng r; memset(&r, 0, sizeof(r));
                    r.state = rng_key(seed, pix, (uint32_t)smp);
                    v3 L = trace_sample(s, backend, cam, W, H, x, y, depth, &r, 0, counters ? loc : NULL);
                    acc[0] = acc[0] + L.x; acc[1] = acc[1] + L.y; acc[2] = acc[2] + L.z;
                }
            }
            out_sum[3 * slot + 0] = acc[0];
            out_sum[3 * slot + 1] = acc[1];
            out_sum[3 * slot + 2] = acc[2];
        }
        if (counters) {
#pragma omp critical
            for (int k = 0; k < 4; ++k) tot[k] += loc[k];
        }
    }
    if (counters) for (int k = 0; k < 4; ++k) counters[k] = tot[k];
    return 0;
}
