#pragma once
// prt_kernels.hip — the per-ray path-tracing hot path for CDNA4 (gfx950).
//
// One persistent kernel runs PathTracer.trace (reference core/tracing.py:116-155)
// for every (pixel, sample) work item of a tile set.  Each 64-lane wave owns a
// work queue (chunks pulled from one device counter, handed to idle lanes with
// __ballot / popcount ranks — path regeneration), and every loop iteration runs
// exactly ONE ray query per active lane: either a closest-hit extension ray or
// an any-hit NEE shadow ray.  Lanes therefore stay busy across paths of
// different length, and both query kinds share one traversal loop.
//
// Arithmetic contract (shared with oracle/prt_oracle.c):
//   f32, no FMA contraction (-ffp-contract=off and the pragma below),
//   correctly rounded '/' and sqrtf (hipcc default on gfx950), expressions in
//   the reference's left-to-right order, the PCG stream of DESIGN.md §RNG and
//   the minimax sin/cos of the concentric map.
// Closest hit = minimal (t, original triangle index); the BVH only prunes.
//
// This header holds the device code of the trace kernel; it is compiled once per
// (traversal stack, stats) instantiation set (prt_trace_inst.hip, in parallel) and
// by prt_kernels.hip for the hit-query, camera and reduction kernels.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "prt_kernels.h"

namespace prt {
namespace {

constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kPiOver4 = 0.78539816339744830961f;
constexpr float kTMin = 0.00001f;    // core/tracing.py:127
constexpr float kTMax = 99999.9f;    // core/tracing.py:127
constexpr float kGamma = 0x1.000006p+0f;  // f32(1 + 2*GAMMA2_3), bvh_taichi.py:179
constexpr int kBlock = 256;
constexpr int kChunk = 64;           // work items per queue refill (one atomic)

struct V3 { float x, y, z; };
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// a / b is NaN (IEEE): a or b NaN, 0/0 or inf/inf
__device__ __forceinline__ bool div_is_nan(float a, float b) {
    return isnan(a) || isnan(b) || (a == 0.0f && b == 0.0f) || (isinf(a) && isinf(b));
}
// (a.x / b, a.y / b, a.z / b), correctly rounded like IEEE division.  The compiler's
// expansion of one f32 division on gfx950 is
//     v_div_scale (den), v_rcp, 2 fma (reciprocal refinement), v_div_scale (num), mul,
//     3 fma (two quotient corrections, the last as v_div_fmas), v_div_fixup
// and v_div_scale / v_div_fixup change nothing when numerator and denominator are finite
// with |x| in [2^-40, 2^40]: the exponent difference (<= 80) stays below the scaling
// threshold of 96, the denominator, its reciprocal and the quotient are normal, and the
// numerator's biased exponent exceeds 23.  For such operands the remaining sequence
// is therefore bit-identical to the full expansion, and the reciprocal refinement is
// shared by the three quotients of one denominator.  A wave with any lane outside the
// range (zero, tiny, huge, inf, NaN) takes the plain divisions.
// fminf drops a NaN operand, the sum does not: a NaN or inf anywhere fails `sum <= 2^40`
__device__ __forceinline__ bool div3_fast_ok(V3 a, float b) {
    const float lo = fminf(fminf(fabsf(a.x), fabsf(a.y)), fminf(fabsf(a.z), fabsf(b)));
    const float sum = (fabsf(a.x) + fabsf(a.y)) + (fabsf(a.z) + fabsf(b));
    return lo >= 0x1p-40f && sum <= 0x1p40f;
}
__device__ __forceinline__ V3 div3_fast(V3 a, float b) {
    float r = __builtin_amdgcn_rcpf(b);
    r = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
    auto q1 = [&](float n) {
        float q = n * r;
        q = __builtin_fmaf(__builtin_fmaf(-b, q, n), r, q);
        return __builtin_fmaf(__builtin_fmaf(-b, q, n), r, q);
    };
    return v3(q1(a.x), q1(a.y), q1(a.z));
}
__device__ __forceinline__ V3 div3(V3 a, float b) {
    if (__ballot(!div3_fast_ok(a, b)) == 0) return div3_fast(a, b);
    return v3(a.x / b, a.y / b, a.z / b);
}
// (a.x / pdf, a.y / pdf, a.z / pdf) under the reference's NaN rule (tracing.py:146-148): when
// any quotient would be NaN, pdf = 1e-4 instead.  Operands in div3's fast range (finite,
// magnitudes in [2^-40, 2^40]) cannot give a NaN quotient, so a wave whose lanes are all in
// range skips the NaN tests.
__device__ __forceinline__ V3 div3_nan_guard(V3 a, float pdf) {
    if (__ballot(!div3_fast_ok(a, pdf)) == 0) return div3_fast(a, pdf);
    if (div_is_nan(a.x, pdf) || div_is_nan(a.y, pdf) || div_is_nan(a.z, pdf)) pdf = 1e-4f;
    return v3(a.x / pdf, a.y / pdf, a.z / pdf);
}
// v_cmp_class_f32 masks (one VALU instruction tests any set of IEEE classes)
constexpr int kClassNegNormal = 1 << 3, kClassPosZero = 1 << 6, kClassPosNormal = 1 << 8;
constexpr int kClassNormal = kClassNegNormal | kClassPosNormal;
constexpr int kClassDenorm = (1 << 4) | (1 << 7);
// 1 / b, correctly rounded: for finite |b| in [2^-40, 2^40] the division expansion (see
// div3) with numerator 1 is the refined reciprocal plus two quotient corrections
// (its q = 1 * r is exact).
// the sequence itself (prt_selftest_rcp / prt_selftest_guards compare it with the IEEE division
// over all 2^32 floats)
__device__ __forceinline__ float rcp_fast_seq(float b) {
    float r = __builtin_amdgcn_rcpf(b);
    r = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
    const float q = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
    return __builtin_fmaf(__builtin_fmaf(-b, q, 1.0f), r, q);
}
// The wave's lanes of class mask m, as one v_cmp_class_f32 into an SGPR pair (inactive lanes read 0).
// Written out because the ballot of llvm.amdgcn.class is lowered through a VGPR (v_cndmask + v_cmp: two
// more VALU per test), and the mask sits in an SGPR (above 64 it is no inline constant; a VGPR copy
// pinned across the loops cost the pooled kernel a spill).
__device__ __forceinline__ uint64_t class_lanes(float x, int m) {
    uint64_t k;
    asm("v_cmp_class_f32_e64 %0, %1, %2" : "=s"(k) : "v"(x), "s"(m));
    return k;
}
// rcp_fast_seq's guard, on the RESULT (round 6): whenever the sequence returns a
// normal float it returns 1.0f / b — proven by the exhaustive sweep over all 2^32 operands on gfx950
// (prt_selftest_guards counter 0 with this per-lane form, tests/test_gpu_selftest.py); zero, denormal,
// huge (> 2^126), infinite and NaN operands give a non-normal result and take the division.  One
// v_cmp_class per test instead of round 5's two range compares on |b|.
__device__ __forceinline__ bool rcp_guard_ok(float r) { return __builtin_amdgcn_classf(r, kClassNormal); }
__device__ __forceinline__ float rcp_exact(float b) {
    float r = rcp_fast_seq(b);
    if (class_lanes(r, kClassNormal) != __builtin_amdgcn_read_exec()) {
        // a real branch: without the (empty, volatile) asm the compiler if-converts the division into
        // every test (both sequences and a select); a non-inlined division here (a cold call) ran 0.2 %
        // slower at C2 (profiles/r06/guards/)
        asm volatile("");
        r = 1.0f / b;
    }
    return r;
}
// Correctly rounded sqrt.  hipcc expands sqrtf on gfx950 as: scale x by 2^32 when
// x < 2^-96, v_sqrt_f32, correct the result by one ulp down / up from the signs of the
// residuals fma(-(s -/+ 1 ulp), s, x), unscale, and return x itself for +-0 / +inf.  With FAST
// a wave whose operands are all in the guard's domain (below) runs the corrected v_sqrt alone
// (bit-identical); other waves take sqrtf.  FAST is used by the LDS-scene kernels (C2 -0.5 %); the
// global-scene kernel keeps sqrtf (its extra live registers cost spills there).
// the sequence itself (prt_selftest_guards sweeps it over all 2^32 floats against sqrtf)
__device__ __forceinline__ float sqrt_fast_seq(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u);
    const float su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x);
    const float ru = __builtin_fmaf(-su, s, x);
    const float r = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : r;
}
// Its guard (round 6): x >= 2^-96, ONE compare instead of round 5's range test
// [2^-96, FLT_MAX].  The exhaustive sweep over all 2^32 floats (prt_selftest_guards counters 4-9)
// finds the sequence equal to sqrtf for every operand except the denormals (of either sign) and the
// operands in [+0, 2^-96), where sqrtf scales: +inf gives +inf on both sides, negative operands and NaN
// give NaN on both sides, so the upper bound was never needed.
__device__ __forceinline__ bool sqrt_guard_ok(float x) { return x >= 0x1p-96f; }
template <bool FAST>
__device__ __forceinline__ float sqrt_cr(float x) {
    if constexpr (FAST) {
        if (__ballot(!sqrt_guard_ok(x)) == 0) return sqrt_fast_seq(x);
        asm volatile("");
    }
    return sqrtf(x);
}
// taichi_glsl normalize: v / length(v) (IEEE division, correctly rounded sqrt).
// FAST (round 6): the shared-reciprocal quotients under a cheaper guard than div3's — every |a_i| >=
// 2^-60 and s = length(a) <= 2^64 (four compares, no min / sum chain).  That is
// div3's no-scaling condition for this quotient: s >= |a_i| (1 - 2^-23) > 2^-61 (s = sqrt(dot) and
// dot >= each rounded square), so s and 1/s are normal, |a_i / s| <= 1 + 2^-23 (no overflow, exponent
// difference <= 1 < 96), |a_i / s| >= 2^-124 (normal with two binades of margin), every a_i has a
// biased exponent >= 67 > 23 and none is zero; an infinite a_i makes s infinite and a NaN fails its
// compare, so those waves divide.
template <bool FAST = false>
__device__ __forceinline__ V3 normalize(V3 a) {
    const float s = sqrt_cr<FAST>(dot(a, a));
    if constexpr (FAST) {
        const bool ok = (int)(fabsf(a.x) >= 0x1p-60f) & (int)(fabsf(a.y) >= 0x1p-60f) &
                        (int)(fabsf(a.z) >= 0x1p-60f) & (int)(s <= 0x1p64f);
        if (__ballot(!ok) == 0) return div3_fast(a, s);
        return v3(a.x / s, a.y / s, a.z / s);
    }
    return div3(a, s);
}
__device__ __forceinline__ V3 xyz(float4 f) { return v3(f.x, f.y, f.z); }
// The Lambert vertex's BRDF weight division (att * max(cw, 0)) / (|cw| / pi) under the reference's NaN
// rule (tracing.py:146-148; ad = att * dz, pdf = |cw| * InvPi).  FAST (round 6):
// on a scene whose albedos lie in [2^-40, 2^40] and whose face normals have length in [0.5, 2]
// (TraceParams::shade_fast, checked on the host), cw >= 2^-60 alone puts the quotient in div3's
// no-scaling domain: cw <= |n| |wi| <= 2 (wi normalised; sphere normals (p - c) / r ~ 1), so pdf =
// cw / pi is normal in [2^-62, 1], ad_i = att_i cw in [2^-100, 2^41] (normal, biased exponent >= 27 >
// 23, non-zero), ad_i / pdf ~ pi att_i in [2^-39, 2^42] (normal, exponent difference <= 42 < 96), and
// no quotient is NaN, so the rule does not fire: one compare instead of div3's range test (a NaN cw
// fails it).
template <bool FAST>
__device__ __forceinline__ V3 lambert_div(V3 ad, float pdf, float cw, int shade_fast) {
    if constexpr (FAST) {
        if (shade_fast && __ballot(!(cw >= 0x1p-60f)) == 0) return div3_fast(ad, pdf);
    }
    return div3_nan_guard(ad, pdf);
}
// The NEE term's division (em * dot1 * dot2) / |p - p2|^2 (tracing.py:92-108).  FAST (round 6): under
// shade_fast (above) em_i in [2^-40, 2^40] and dot1, dot2 <= 2 (unit-ish w, normals of length <= 2), so
// with dot1, dot2 >= 2^-20 and sl in [2^-40, 2^40] the numerators lie in [2^-81, 2^42] (normal, biased
// exponent >= 46), sl and 1 / sl are normal, the quotients lie in [2^-121, 2^82] and the exponent
// difference is <= 82 < 96: div3's no-scaling domain with four compares instead of div3's range test.
template <bool FAST>
__device__ __forceinline__ V3 nee_div(V3 a, float sl, float dot1, float dot2, int shade_fast) {
    if constexpr (FAST) {
        const bool ok = (int)(dot1 >= 0x1p-20f) & (int)(dot2 >= 0x1p-20f) & (int)(sl >= 0x1p-40f) &
                        (int)(sl <= 0x1p40f);
        if (shade_fast && __ballot(!ok) == 0) return div3_fast(a, sl);
    }
    return div3(a, sl);
}


// ------------------------------------------------------------------ RNG spec
__device__ __forceinline__ uint32_t pcg_permute(uint32_t s) {
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) { return pcg_permute(v * 747796405u + 2891336453u); }
__device__ __forceinline__ uint32_t rng_key(uint32_t seed_lo, uint32_t seed_hi, uint32_t pixel, uint32_t sample) {
    uint32_t h = pcg_hash(seed_lo);
    h = pcg_hash(h ^ seed_hi ^ pixel);
    return pcg_hash(h + sample);
}
__device__ __forceinline__ float rng_next(uint32_t& st) {
    st = st * 747796405u + 2891336453u;
    return (float)(pcg_permute(st) >> 8) * 0x1p-24f;
}
// taichi_glsl randInt(a, b), inclusive
__device__ __forceinline__ int rng_int(uint32_t& st, int a, int b) {
    float u = rng_next(st);
    int k = (int)floorf(u * (float)(b - a + 1));
    k = k > b - a ? b - a : k;
    return a + k;
}

// --------------------------------------------- concentric disk (samplers.py:9-32)
__device__ __forceinline__ float poly_sin(float x) {
    float z = x * x;
    return ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x + x;
}
__device__ __forceinline__ float poly_cos(float x) {
    float z = x * x;
    return ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
           - 0.5f * z + 1.0f;
}
template <bool FAST = false>
__device__ __forceinline__ V3 cosine_hemisphere(float u0, float u1) {
    float ox = 2.0f * u0 - 1.0f, oy = 2.0f * u1 - 1.0f;
    float dx = 0.0f, dy = 0.0f;
    if (!(ox == 0.0f && oy == 0.0f)) {
        // |ox| > |oy|: r = ox, theta = pi/4 (oy/ox), (c, s) = (cos, sin)(theta);
        // else:        r = oy, a = pi/4 (ox/oy), theta = pi/2 - a, (c, s) = (sin, cos)(a).
        // Both cases as one division and one polynomial pair on selected operands (a
        // divergent if/else would run two of each on a wave holding both cases).
        const bool wide = fabsf(ox) > fabsf(oy);
        const float r = wide ? ox : oy;
        float t;
        if constexpr (FAST) {
            // round 6: the quotient by div3's shared-reciprocal sequence, unguarded: u0, u1 are
            // rng_next draws (multiples of 2^-24 in [0, 1)), so ox, oy = 2u - 1 are exact multiples of
            // 2^-23 in [-1, 1): |r| >= 2^-23 and the numerator is +0 or of magnitude in [2^-23, |r|] —
            // div3's no-scaling domain (quotient in [2^-23, 1], biased exponents >= 104), and for
            // the numerator +0 the sequence returns the IEEE zero of sign(r) itself
            const float q = wide ? oy : ox;
            float rr = __builtin_amdgcn_rcpf(r);
            rr = __builtin_fmaf(__builtin_fmaf(-r, rr, 1.0f), rr, rr);
            float qq = q * rr;
            qq = __builtin_fmaf(__builtin_fmaf(-r, qq, q), rr, qq);
            t = kPiOver4 * __builtin_fmaf(__builtin_fmaf(-r, qq, q), rr, qq);
        } else {
            t = kPiOver4 * ((wide ? oy : ox) / r);
        }
        const float pc = poly_cos(t), ps = poly_sin(t);
        dx = r * (wide ? pc : ps);
        dy = r * (wide ? ps : pc);
    }
    float m = 1.0f - dx * dx - dy * dy;
    return v3(dx, dy, sqrt_cr<FAST>(m > 0.0f ? m : 0.0f));
}

// rotate_z_to + rotate_vector (mat4_taichi.py:9-60): rows (x, z, n)
__device__ __forceinline__ V3 to_world(V3 n, V3 l) {
    V3 v = normalize(n);
    V3 r1, r2, r3;
    if (v.y == 1.0f) {
        r1 = v3(1, 0, 0); r2 = v3(0, 0, 1); r3 = v3(0, 1, 0);
    } else if (v.y == -1.0f) {
        r1 = v3(1, 0, 0); r2 = v3(0, 0, 1); r3 = v3(0, -1, 0);
    } else {
        V3 x = normalize(cross(v, v3(0.0f, 1.0f, 0.0f)));
        V3 z = normalize(cross(x, v));
        r1 = x; r2 = z; r3 = v;
    }
    return normalize(r1 * l.x + r2 * l.y + r3 * l.z);
}

// ------------------------------------------------------- camera (camera_taichi.py:47-74)
__device__ __forceinline__ void gen_ray(const float* cam, float u, float v, uint32_t& st, V3& o, V3& d) {
    const float sd0 = cam[16], sd1 = cam[17], sd2 = cam[18], sd3 = cam[19];
    float rd[4] = {(u - 0.5f) * sd0 / 0.5f, (v - 0.5f) * sd1 / 0.5f, -sd2, 1.0f};
    float ro[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    if (sd3 > 0.0f) {
        ro[0] = sd2 * rng_next(st) - sd2 / 2.0f;
        ro[1] = sd2 * rng_next(st) - sd2 / 2.0f;
    }
    float dw[4], ow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float* c = cam + 4 * i;
        dw[i] = rd[0] * c[0] + rd[1] * c[1] + rd[2] * c[2] + rd[3] * c[3];
        ow[i] = ro[0] * c[0] + ro[1] * c[1] + ro[2] * c[2] + ro[3] * c[3];
    }
    float f0 = dw[0] - ow[0], f1 = dw[1] - ow[1], f2 = dw[2] - ow[2], f3 = dw[3] - ow[3];
    float l = sqrtf(f0 * f0 + f1 * f1 + f2 * f2 + f3 * f3);
    o = v3(ow[0], ow[1], ow[2]);
    d = v3(f0 / l, f1 / l, f2 / l);
}

// -------------------------------------- specular helpers (bsdf_taichi.py:6-22)
__device__ __forceinline__ float schlick(float cosine, float idx) {
    float r0 = (1.0f - idx) / (1.0f + idx);
    r0 = r0 * r0;
    float m = 1.0f - cosine;
    return r0 + (1.0f - r0) * (m * m * m * m * m);
}
__device__ __forceinline__ V3 reflect3(V3 v, V3 n) { return v - n * (2.0f * dot(v, n)); }
__device__ __forceinline__ V3 refract3(V3 v, V3 n, float eta) {
    float ct = -dot(v, n);
    ct = ct > 1.0f ? 1.0f : ct;
    V3 perp = (v + n * ct) * eta;
    float k = 1.0f - dot(perp, perp);
    return perp + n * (-sqrtf(fabsf(k)));
}
// random_in_unit_sphere (vec3_taichi.py:299-306) with deterministic ops: see oracle
__device__ __forceinline__ float cbrt_spec(float x) {
    if (!(x > 0.0f)) return 0.0f;
    float y = __uint_as_float(__float_as_uint(x) / 3u + 709921077u);
    for (int i = 0; i < 3; ++i) y = (2.0f * y + x / (y * y)) / 3.0f;
    return y;
}
__device__ __forceinline__ V3 random_in_unit_sphere(uint32_t& st) {
    float u1 = rng_next(st), u2 = rng_next(st), u3 = rng_next(st);
    int q = (int)floorf(u1 * 4.0f + 0.5f);
    float a = 6.28318530717958647692f * (u1 - 0.25f * (float)q);
    float pc = poly_cos(a), ps = poly_sin(a);
    float c, sn;
    switch (q & 3) {
        case 0: c = pc; sn = ps; break;
        case 1: c = -ps; sn = pc; break;
        case 2: c = -pc; sn = -ps; break;
        default: c = ps; sn = -pc; break;
    }
    float z = 2.0f * u2 - 1.0f;
    float m = 1.0f - z * z;
    float sp = sqrtf(m > 0.0f ? m : 0.0f);
    float r = cbrt_spec(u3);
    return v3(r * sp * c, r * sp * sn, r * z);
}
// hit_sphere (intersection_taichi.py:15-36): nearest root in [t_min, t_max], else far root
__device__ __forceinline__ bool sphere_hit(float4 sc, V3 o, V3 d, float t_min, float t_max, float& root) {
    V3 oc = o - xyz(sc);
    float a = dot(d, d);
    float half_b = dot(oc, d);
    float cc = dot(oc, oc) - sc.w * sc.w;
    float disc = half_b * half_b - a * cc;
    if (!(disc >= 0.0f)) return false;
    float sq = sqrtf(disc);
    root = (-half_b - sq) / a;
    if (root < t_min || t_max < root) {
        root = (-half_b + sq) / a;
        if (root < t_min || t_max < root) return false;
    }
    return true;
}

// ---------------------------------------------------------------- traversal
struct Counters {
    uint32_t nodes, tris, ext, shadow, it_inner, it_leaf, max_sp, nonfinite, w_tri, q0, max_q;
    // STATS lane table (trace_kernel_pool, diag words 160..): wave-level trips of the traversal's
    // inner-node and triangle loops, and the active lanes summed over those trips (wave_tick)
    uint32_t wi, li, wl, ll;
};
// STATS: one wave-level trip of the enclosing loop body, booked by its first active lane, with
// the lanes active in it: sum(l) / (64 sum(w)) is that loop's SIMD lane utilisation
__device__ __forceinline__ void wave_tick(uint32_t& w, uint32_t& l) {
    const uint32_t pc = (uint32_t)__popcll(__ballot(true));
    if ((uint32_t)__builtin_amdgcn_readfirstlane(__lane_id()) == __lane_id()) { w += 1u; l += pc; }
}

// Moller-Trumbore in the reference's exact expression order
// (intersection_taichi.py:69-91), for closest-hit and any-hit lanes of one wave.
// nodes/tris point either to global memory or to the block's LDS copy of a
// small scene (the compiler infers the address space after inlining).
__device__ __forceinline__ bool mt_u(V3 v0, V3 e1, V3 e2, V3 o, V3 d, float t0, float tbest, int id, int best_id,
                                     bool any, float& tout) {
    // branch-free: a lane failing an early test would wait for the wave's other lanes
    // anyway, so every value is computed and the tests are combined (same results as the
    // reference's early returns; det == 0 is rejected, its quotient never used)
    V3 c = cross(e1, d);
    float det = dot(c, e2);
    const bool nz = fabsf(det) > 0.0f;
    float f = rcp_exact(det);   // det == 0 takes rcp_exact's division (inf): masked by nz below
    V3 s = o - v0;
    V3 q = cross(s, e2);
    float t = -f * dot(q, e1);
    float u = -f * dot(q, d);
    float v = f * dot(c, s);
    // bitwise (not short-circuit) combination: one lane mask, no exec-mask branches
    const bool in_range = (t0 < t) & ((t < tbest) | ((!any) & (t == tbest) & (id < best_id)));
    const bool hit = nz & in_range & (0.0f <= u) & (u <= 1.0f) & (v >= 0.0f) & (1.0f - u - v >= 0.0f);
    tout = t;
    return hit;
}

// While-while traversal (Aila & Laine 2009, "persistent while-while"): lanes
// descend inner nodes until every lane of the wave holds a postponed leaf,
// then all lanes test leaf triangles together, so inner-node and leaf work
// of different lanes do not serialise against each other.  Stack bottom
// holds kSentinel; leaves are negative references, inner nodes >= 0.
constexpr int kSentinel = 0x7FFFFFFF;
constexpr uint32_t kGuardTrips = 1u << 20;   // leaf batches per query before the watchdog trips

// While-while over the BVH4 (prt_internal.h): one node fetch tests four child
// boxes; the nearest hit child is visited next (a 3-comparator tournament) and the
// other hit children are pushed.

// Per-lane traversal stacks.  LdsStack: entry k at l[k * kBlock] (conflict-free).
// SpillStack: the first LST entries in LDS, deeper ones in a per-lane global area
// (stride = all threads of the grid); deep stacks are rare (max 24 entries measured on
// the 1 M-triangle scene against a worst-case bound of 46), so a small LDS stack keeps
// occupancy and the spill branch is almost never taken.
struct LdsStack {
    static constexpr int kSent = kSentinel;
    static constexpr int kStep = 1;   // sp advances by kStep per entry (LdsStack16A: bytes)
    int* l;
    __device__ __forceinline__ int origin() const { return 0; }
    __device__ __forceinline__ int depth(int sp) const { return sp; }
    __device__ __forceinline__ void put(int k, int v) { l[k * kBlock] = v; }
    __device__ __forceinline__ int get(int k) const { return l[k * kBlock]; }
    // entries [0, k] of every lane are in LDS (always)
    __device__ __forceinline__ bool lds_only(int) const { return true; }
    __device__ __forceinline__ LdsStack lds() const { return *this; }
};
template <int LST>
struct SpillStack {
    static constexpr int kSent = kSentinel;
    static constexpr int kStep = 1;
    int* l;
    __device__ __forceinline__ int origin() const { return 0; }
    __device__ __forceinline__ int depth(int sp) const { return sp; }
    int* g;
    uint32_t gs;
    __device__ __forceinline__ void put(int k, int v) {
        if (k < LST) l[k * kBlock] = v;
        else g[(size_t)(k - LST) * gs] = v;
    }
    __device__ __forceinline__ int get(int k) const { return k < LST ? l[k * kBlock] : g[(size_t)(k - LST) * gs]; }
    // wave-uniform: no lane touches an entry above k < LST, so the spill branches can go
    __device__ __forceinline__ bool lds_only(int k) const { return __ballot(k >= LST) == 0; }
    __device__ __forceinline__ LdsStack lds() const { return LdsStack{l}; }
};
// LDS-resident scenes: 16-bit entries (half the stack's LDS, so the octant node copies
// fit beside it at six blocks per CU).  Node indices and leaf references of such scenes fit
// 16 bits (host check in lds_fits4), and the traversal sentinel is 0x7FFF: the block's LDS
// copy of the BVH4 rewrites the empty-slot references to it.  Entry k of lane j sits at
// 2 * (k * kBlock + (j & ~63) + 2 * (j & 31) + (j >> 5 & 1)): a half-wave's 32 lanes use 32
// different banks.
struct LdsStack16 {
    static constexpr int kSent = 0x7FFF;
    static constexpr int kStep = 1;
    short* l;
    __device__ __forceinline__ int origin() const { return 0; }
    __device__ __forceinline__ int depth(int sp) const { return sp; }
    __device__ __forceinline__ void put(int k, int v) { l[k * kBlock] = (short)v; }
    __device__ __forceinline__ int get(int k) const { return (int)l[k * kBlock]; }
    __device__ __forceinline__ bool lds_only(int) const { return true; }
    __device__ __forceinline__ LdsStack16 lds() const { return *this; }
};
// LdsStack16 with the stack pointer held as the entry's LDS byte ADDRESS (round 6): a push writes at
// sp + kStep as an immediate offset of the pointer register and advances it by a select, a pop reads at
// sp — no per-entry address arithmetic (the index form spends a v_lshl_add on every push and pop:
// three or four per node visit)
typedef __attribute__((address_space(3))) short LdsShort;
struct LdsStack16A {
    static constexpr int kSent = 0x7FFF;
    static constexpr int kStep = 2 * kBlock;
    int base;   // LDS byte address of this lane's entry 0
    __device__ __forceinline__ void put(int k, int v) { *(LdsShort*)(uintptr_t)(uint32_t)k = (short)v; }
    __device__ __forceinline__ int get(int k) const { return (int)*(const LdsShort*)(uintptr_t)(uint32_t)k; }
    __device__ __forceinline__ int origin() const { return base; }
    __device__ __forceinline__ int depth(int sp) const { return (sp - base) / kStep; }
    __device__ __forceinline__ bool lds_only(int) const { return true; }
    __device__ __forceinline__ LdsStack16A lds() const { return *this; }
};
// sp advanced by one entry where p holds.  Address form: the 0 / 1 select laundered into a register and
// shifted by the entry stride (one v_cndmask + one v_lshl_add); as a select of 0 / 512 the stride would
// need a VGPR of its own (gfx950 reads one scalar operand per VALU instruction besides the mask), which
// the pooled kernel pays with spills
template <class S>
__device__ __forceinline__ int stack_adv(int sp, bool p) {
    if constexpr (S::kStep == 1) {
        return sp + (p ? 1 : 0);
    } else {
        int b = p ? 1 : 0;
        asm volatile("" : "+v"(b));
        return sp + (b << __builtin_ctz(S::kStep));
    }
}

// MODE 0: per-lane query kind (`any` may differ between lanes); 1: every lane
// closest-hit; 2: every lane any-hit (phase-aligned shadow iterations).  Any-hit
// queries need no visiting order, so mode 2 skips the sorting network.
// Pushes write the slot above the top unconditionally and advance the stack
// pointer by the hit predicate (no exec-mask branches); the highest slot written
// is the same as with conditional pushes (<= 3 above the entry top).
// LDS-resident scene data (the block's octant node copies and triangles) addressed as LDS: the
// element offset stays a 32-bit LDS address (v_mad_u32_u24 / v_lshl_add) instead of the 64-bit
// flat-pointer arithmetic (v_mad_u64_u32) the generic pointer gets before address-space inference
typedef float F4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const F4v LdsF4;
__device__ __forceinline__ const LdsF4* as_lds(const float4* p) { return (const LdsF4*)p; }
// one ds_read_b128 of element i
__device__ __forceinline__ float4 lds4(const LdsF4* p, int i) {
    const F4v v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

// Slab test from plane distances already ordered near/far (quantised nodes).
__device__ __forceinline__ bool slab_t(float nx, float fx, float ny, float fy, float nz, float fz, float tmin,
                                       float tmax, float& tn) {
    float tnear = fmaxf(fmaxf(nx, ny), fmaxf(nz, tmin));
    float tfar = fminf(fminf(fx, fy), fminf(fz, tmax)) * kGamma;
    tn = tnear;
    return tnear <= tfar;
}
__device__ __forceinline__ float ubyte(uint32_t w, int k) {
    return (float)((w >> (8 * k)) & 0xFFu);   // v_cvt_f32_ubyte{k}
}
// Child k of a quantised node (prt_internal.h): plane distance (origin + q s - o) / d
// evaluated as fma(q, s/d, (origin - o)/d); the >= 2 pad outward rounding of the grid
// covers the estimate's error, so the test stays conservative.  The q words arrive
// already swapped into near/far order by the sign of 1/d (see slab_nf()).
struct QAxis { float A, B; };
__device__ __forceinline__ bool qchild(int k, uint32_t lxq, uint32_t hxq, uint32_t lyq, uint32_t hyq, uint32_t lzq,
                                       uint32_t hzq, QAxis X, QAxis Y, QAxis Z, float tmin, float tmax, float& tn) {
    return slab_t(__builtin_fmaf(ubyte(lxq, k), X.A, X.B), __builtin_fmaf(ubyte(hxq, k), X.A, X.B),
                  __builtin_fmaf(ubyte(lyq, k), Y.A, Y.B), __builtin_fmaf(ubyte(hyq, k), Y.A, Y.B),
                  __builtin_fmaf(ubyte(lzq, k), Z.A, Z.B), __builtin_fmaf(ubyte(hzq, k), Z.A, Z.B), tmin, tmax, tn);
}

// Traversal state of a query that may be suspended between loop iterations (RES).
struct TState { int cur, leaf, sp, best_id; float best; };
// A query whose t_max is NaN (the reference's shadow bound t_at_light = (p2.x - p.x) / w.x
// is 0/0 when p2.x == p.x, core/tracing.py:97) can never accept a triangle: Moller-Trumbore
// needs t < t_max (intersection_taichi.py:84), false against NaN.  Its slab tests never cull
// either (fminf drops the NaN), so traversing would walk every box along the whole line
// (config 4: ~2000 node visits, the launch's last 2 ms); it starts finished instead, with
// the same (miss) result.  Spheres still see the NaN bound (hit_sphere accepts it).
template <class S>
__device__ __forceinline__ int root_for(float tmax) { return tmax == tmax ? 0 : S::kSent; }

template <class S>
__device__ __forceinline__ void tstate_init(TState& ts, S stk, float tmax) {
    stk.put(stk.origin(), S::kSent);
    ts.cur = root_for<S>(tmax); ts.leaf = 0; ts.sp = stk.origin(); ts.best_id = -1; ts.best = tmax;
}

// RES: the wave leaves the traversal loop once fewer than `min_lanes` lanes are still
// traversing; the unfinished lanes keep their state (registers + LDS stack) and resume
// in the next iteration, so the long tail of a few slow lanes no longer idles the
// others.  Returns whether the query finished (hit_id / hit_t valid).
// Conservative slab test on a padded box (PBRT-style 1+2*gamma3 on t_far).
// t = (lo - o) / d is evaluated as fma(lo, 1/d, -o/d): pruning only, so the few-ulp
// error of the estimate is covered by the box padding (~1e-6 of the scene scale,
// >> |o/d| ulp) and the 1+2*gamma3 factor on t_far.  The near and far plane of each
// axis are chosen by the sign of 1/d, NOT by min/max of the two distances: for a
// direction component of exactly 0 (1/d = inf) a plane distance can be NaN, and
// fminf/fmaxf would then turn the other plane's -inf into the FAR distance and cull
// a box the ray lies inside (measured: 8 of 262144 pixels at config 2).  With the
// selection, a NaN distance is dropped by the fmaxf/fminf that follow, which can
// only enlarge the interval.  For f32 BVH4 nodes the selection is an address offset
// (no per-plane selects); quantised nodes swap their plane words (qchild).
__device__ __forceinline__ bool slab_nf(float nx, float fx, float ny, float fy, float nz, float fz, V3 oi, V3 inv,
                                        float tmin, float tmax, float& tn) {
    float ax = __builtin_fmaf(nx, inv.x, -oi.x), bx = __builtin_fmaf(fx, inv.x, -oi.x);
    float ay = __builtin_fmaf(ny, inv.y, -oi.y), by = __builtin_fmaf(fy, inv.y, -oi.y);
    float az = __builtin_fmaf(nz, inv.z, -oi.z), bz = __builtin_fmaf(fz, inv.z, -oi.z);
    float tnear = fmaxf(fmaxf(ax, ay), fmaxf(az, tmin));
    // the reference's 1 + 2 gamma_3 factor on t_far (bvh_taichi.py:179).  The box padding (1e-6 of
    // the scene's largest coordinate, ~8 ulps) alone would keep the test conservative, and dropping the
    // factor saves 4 VALU per visit (-D PRT_SLAB_GAMMA=0: C2 3.873 vs 3.884, C3 70.75 vs 71.14 ms per
    // launch, images identical), but the pooled kernel then spills 3 VGPRs and writes 0.14 GB more
    // per frame to HBM (profiles/r05/gamma/): kept
#ifndef PRT_SLAB_GAMMA
#define PRT_SLAB_GAMMA 1
#endif
    // (fminf canonicalises the loop-carried tmax, one VALU per visit; an asm v_min_f32 without it pins
    // registers: 7 spilled VGPRs, C2 +0.6 %, profiles/r06/guards/)
    float tfar = fminf(fminf(bx, by), fminf(bz, tmax));
    if (PRT_SLAB_GAMMA) tfar *= kGamma;
    tn = tnear;
    return tnear <= tfar;
}

// Slab reciprocals 1/d, clamped to +-1e30.  A direction component of exactly +-0 (one cosine
// draw in 2^24) would give 1/d = +-inf, and fma(plane, 1/d, -o/d) = inf - inf = NaN: the
// near/far selection then drops that axis and the ray culls nothing along it, walking every
// box it overlaps in the other two axes (config 4: 1000-2200 node visits for such a query,
// against 25 on average, each one of the launch's slowest paths).  With the clamp the
// distances are +-1e30 (plane - o) up to the rounding of o * 1e30 (|o| 2^-24 1e30), which the
// box padding (>= 1e-6 |o|) covers: the sign is right and the test stays conservative.
__device__ __forceinline__ V3 ray_inv(V3 d) {
    auto c = [](float x) { return __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(x), -1e30f, 1e30f); };
    return v3(c(d.x), c(d.y), c(d.z));
}

// One inner-node visit of the while-while BVH4 traversal: tests the four child boxes of
// node `cur`, continues with the nearest hit child (MODE 2, any-hit: the last hit child,
// no sorting) and pushes the other hit children; pops the stack when none is hit.
// Pushes write the slot above the top unconditionally and advance the stack pointer by
// the hit predicate (no exec-mask branches); the highest slot written is the same as
// with conditional pushes (<= 3 above the entry top).
// OCT (LDS-resident scenes): `nodes` is the block's octant copy of the BVH4 (8 copies of each
// node, copy k with the near and far planes of each axis pre-arranged for the direction signs
// k = sx | sy << 1 | sz << 2: 7 float4 = nx, fx, ny, fy, nz, fz, refs; node stride 56 float4)
// and `sx` holds the query's copy offset 7 k: the seven reads need no per-plane addresses.
// Copy k also stores the four children in k's front-to-back order, so closest-hit visits of
// an octant copy take the first hit child instead of sorting entry distances (see step).
template <bool STATS, int MODE, class S, bool QN, bool OCT = false>
__device__ __forceinline__ void visit_node4(const float4* __restrict__ nodes, int& cur, int& sp, S stk, V3 inv, V3 oi,
                                            int sx, int sy, int sz, float tmin, float best, Counters& cn,
                                            bool any_lane = false) {
    float t0, t1, t2, t3;
    bool h0, h1, h2, h3;
    int r0, r1, r2, r3;
    if (QN) {
        // 64-B nodes at a 32-bit byte offset from the uniform base (saddr + voffset addressing,
        // no 64-bit address arithmetic): BVH4 nodes < refs / 3 < 2^25, so the offset < 2^31
        const float4* nd = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(nodes) + ((uint32_t)cur << 6));
        float4 a = nd[0], b = nd[1], c = nd[2], rf = nd[3];
        if (STATS) { cn.nodes++; cn.it_inner++; }
        QAxis X = {a.w * inv.x, __builtin_fmaf(a.x, inv.x, -oi.x)};
        QAxis Y = {b.x * inv.y, __builtin_fmaf(a.y, inv.y, -oi.y)};
        QAxis Z = {b.y * inv.z, __builtin_fmaf(a.z, inv.z, -oi.z)};
        uint32_t lxq = __float_as_uint(sx ? b.w : b.z), hxq = __float_as_uint(sx ? b.z : b.w);
        uint32_t lyq = __float_as_uint(sy ? c.y : c.x), hyq = __float_as_uint(sy ? c.x : c.y);
        uint32_t lzq = __float_as_uint(sz ? c.w : c.z), hzq = __float_as_uint(sz ? c.z : c.w);
        r0 = __float_as_int(rf.x); r1 = __float_as_int(rf.y); r2 = __float_as_int(rf.z); r3 = __float_as_int(rf.w);
        h0 = qchild(0, lxq, hxq, lyq, hyq, lzq, hzq, X, Y, Z, tmin, best, t0) && r0 != kSentinel;
        h1 = qchild(1, lxq, hxq, lyq, hyq, lzq, hzq, X, Y, Z, tmin, best, t1) && r1 != kSentinel;
        h2 = qchild(2, lxq, hxq, lyq, hyq, lzq, hzq, X, Y, Z, tmin, best, t2) && r2 != kSentinel;
        h3 = qchild(3, lxq, hxq, lyq, hyq, lzq, hzq, X, Y, Z, tmin, best, t3) && r3 != kSentinel;
    } else {
        float4 nx, fx, ny, fy, nz, fz, rf;
        if (OCT) {
#ifdef PRT_NO_LDS_ADDR32
            const float4* nd = nodes + (uint32_t)cur * 56u + sx;
#else
            const LdsF4* nl = as_lds(nodes) + (int)(__umul24((uint32_t)cur, 56u) + (uint32_t)sx);
            auto nd = [&](int i) { return lds4(nl, i); };
#endif
#ifdef PRT_NO_LDS_ADDR32
            nx = nd[0]; fx = nd[1]; ny = nd[2]; fy = nd[3]; nz = nd[4]; fz = nd[5]; rf = nd[6];
#else
            nx = nd(0); fx = nd(1); ny = nd(2); fy = nd(3); nz = nd(4); fz = nd(5); rf = nd(6);
#endif
        } else {
            // near/far planes picked by address (the node stores lo and hi per axis)
            const float4* nd = nodes + (size_t)cur * 8;
            nx = nd[sx]; fx = nd[1 - sx]; ny = nd[2 + sy]; fy = nd[3 - sy]; nz = nd[4 + sz]; fz = nd[5 - sz];
            rf = nd[6];
        }
        if (STATS) { cn.nodes++; cn.it_inner++; }
        h0 = slab_nf(nx.x, fx.x, ny.x, fy.x, nz.x, fz.x, oi, inv, tmin, best, t0);
        h1 = slab_nf(nx.y, fx.y, ny.y, fy.y, nz.y, fz.y, oi, inv, tmin, best, t1);
        h2 = slab_nf(nx.z, fx.z, ny.z, fy.z, nz.z, fz.z, oi, inv, tmin, best, t2);
        h3 = slab_nf(nx.w, fx.w, ny.w, fy.w, nz.w, fz.w, oi, inv, tmin, best, t3);
        r0 = __float_as_int(rf.x); r1 = __float_as_int(rf.y); r2 = __float_as_int(rf.z); r3 = __float_as_int(rf.w);
    }
    // pushes and the pop below touch entries <= sp + 3: plain LDS accesses when no lane of
    // the wave can reach a spill stack's global part (wave-uniform test; always for LdsStack)
    auto step = [&](auto st) {
        if (OCT && MODE != 2) {
            // closest-hit over an LDS octant copy, whose children are stored in the octant's
            // front-to-back order (trace_kernel's copy loop): continue with the first hit child and
            // push the other hit ones so that they pop in that order — no distance keys and no
            // sorting network (C2 4.50 -> 4.40 ms, C3 41.4 -> 40.4 ms; the closest (t, id) does not
            // depend on the visiting order).  Any-hit queries (MODE 2, below) continue with the
            // LAST hit child: back to front is 4.6 % faster at C2 than front to back for the
            // shadow rays (they end at the light, and an occluder near it ends the query)
            const bool p3 = h3 & (h0 | h1 | h2), p2 = h2 & (h0 | h1), p1 = h1 & h0;
            st.put(sp + S::kStep, r3); sp = stack_adv<S>(sp, p3);
            st.put(sp + S::kStep, r2); sp = stack_adv<S>(sp, p2);
            st.put(sp + S::kStep, r1); sp = stack_adv<S>(sp, p1);
            const int tp = st.get(sp);
            const bool any_hit = h0 | h1 | h2 | h3;
            cur = h0 ? r0 : (h1 ? r1 : (h2 ? r2 : (h3 ? r3 : tp)));
            sp -= any_hit ? 0 : S::kStep;
        } else if (MODE == 2) {
            st.put(sp + S::kStep, r0); sp = stack_adv<S>(sp, h0);
            st.put(sp + S::kStep, r1); sp = stack_adv<S>(sp, h1);
            st.put(sp + S::kStep, r2); sp = stack_adv<S>(sp, h2);
            int top = st.get(sp);
            cur = h3 ? r3 : top;
            sp -= h3 ? 0 : S::kStep;
        } else {
            // nearest hit child first by a 3-comparator tournament on the entry distances
            // (misses count as +inf, a hit's distance is finite); the three others are pushed
            // when hit, i.e. when their key is finite: the loser of each pair, then the loser
            // of the final.  Keys and masks stay floats / lane masks (no 0/1 integers).
            // any-hit lanes of a mixed wave (MODE 0, global scenes): farthest hit child first —
            // keys negated (entry distances are >= tmin > 0; misses stay +inf).  A shadow ray ends
            // at the light, and an occluder near that end ends the query: C4 18.85 -> 18.67 ms
            // (the LDS scenes' shadow iterations go back to front for the same reason, MODE 2)
            if (MODE == 0 && any_lane) { t0 = -t0; t1 = -t1; t2 = -t2; t3 = -t3; }
            const float k0 = h0 ? t0 : INFINITY, k1 = h1 ? t1 : INFINITY;
            const float k2 = h2 ? t2 : INFINITY, k3 = h3 ? t3 : INFINITY;
            const bool m01 = k1 < k0, m23 = k3 < k2;
            const float a = m01 ? k1 : k0, xb = m01 ? k0 : k1;
            const float c = m23 ? k3 : k2, xd = m23 ? k2 : k3;
            const int ra = m01 ? r1 : r0, rb = m01 ? r0 : r1;
            const int rc = m23 ? r3 : r2, rd = m23 ? r2 : r3;
            const bool m = c < a;
            const int rn = m ? rc : ra, rl = m ? ra : rc;
            const float xn = m ? c : a, xl = m ? a : c;
            st.put(sp + S::kStep, rb); sp += xb < INFINITY ? S::kStep : 0;
            st.put(sp + S::kStep, rd); sp += xd < INFINITY ? S::kStep : 0;
            st.put(sp + S::kStep, rl); sp += xl < INFINITY ? S::kStep : 0;
            const int tp = st.get(sp);
            const bool any_hit = xn < INFINITY;
            cur = any_hit ? rn : tp;
            sp -= any_hit ? 0 : S::kStep;
        }
    };
    if (stk.lds_only(sp + 3 * S::kStep)) step(stk.lds());
    else step(stk);
}

template <bool STATS, int MODE, class S, bool QN = false, bool RES = false, bool OCT = false>
__device__ __forceinline__ bool traverse_ww4(const float4* __restrict__ nodes, const float4* __restrict__ tris, V3 o,
                                             V3 d, float tmin, float tmax, bool any_lane, S stk, int& hit_id,
                                             float& hit_t, Counters& cn, TState* tsp = nullptr, int min_lanes = 0,
                                             int* fault = nullptr, int leaf_break = 0, int leaf_exit = 0,
                                             uint32_t guard_lim = kGuardTrips) {
    const bool any = MODE == 0 ? any_lane : MODE == 2;
    const V3 inv = ray_inv(d);
    V3 oi = o * inv;
    // near plane index per axis (0 = lo, 1 = hi) from the sign of 1/d
    int sx = __float_as_int(inv.x) < 0 ? 1 : 0, sy = __float_as_int(inv.y) < 0 ? 1 : 0,
        sz = __float_as_int(inv.z) < 0 ? 1 : 0;
    if (OCT) sx = 7 * (sx | (sy << 1) | (sz << 2));   // octant copy offset (visit_node4)
    TState ts;
    if (RES) ts = *tsp;
    else tstate_init(ts, stk, tmax);
    float best = ts.best;
    int best_id = ts.best_id;
    uint32_t guard = 0;
    int sp = ts.sp;
    int cur = ts.cur;
    int leaf = ts.leaf;
    do {
        while (cur >= 0 && cur != S::kSent) {
            visit_node4<STATS, MODE, S, QN, OCT>(nodes, cur, sp, stk, inv, oi, sx, sy, sz, tmin, best, cn, any);
            if (STATS) wave_tick(cn.wi, cn.li);
            if (STATS) cn.max_sp = max(cn.max_sp, (uint32_t)(stk.depth(sp) + 1));
            if (cur < 0 && leaf >= 0) {   // postpone the leaf, keep descending
                leaf = cur;
                cur = stk.get(sp);
                sp -= S::kStep;
            }
            // leave for the leaf phase once at most `leaf_break` of the lanes still
            // descending have no postponed leaf (0: all of them hold one)
            if (__popcll(__ballot(leaf >= 0)) <= (uint32_t)leaf_break) break;
        }
        while (leaf < 0) {
            int v = -leaf - 1;
            int first = v >> 3, cnt = (v & 7) + 1;
            if (STATS) {
                cn.it_leaf++;
                // wave-level triangle-loop trips of this leaf trip (max leaf size over the lanes)
                int mc = 8;
                while (mc > 1 && !__ballot(cnt >= mc)) --mc;
                if (__builtin_amdgcn_readfirstlane(__lane_id()) == __lane_id()) cn.w_tri += mc;
            }
            for (int k = 0; k < cnt; ++k) {
                float4 q0, q1, q2;
#ifndef PRT_NO_LDS_ADDR32
                if constexpr (OCT) {
                    const LdsF4* tp = as_lds(tris) + (int)__umul24((uint32_t)(first + k), 3u);
                    q0 = lds4(tp, 0); q1 = lds4(tp, 1); q2 = lds4(tp, 2);
                } else
#endif
                {
                    const float4* tp = tris + (size_t)(first + k) * 3;
                    q0 = tp[0]; q1 = tp[1]; q2 = tp[2];
                }
                int id = __float_as_int(q0.w);
                float t;
                if (STATS) { cn.tris++; wave_tick(cn.wl, cn.ll); }
                if (mt_u(xyz(q0), xyz(q1), xyz(q2), o, d, tmin, best, id, best_id, any, t)) {
                    best = t;
                    best_id = id;
                    if (any) { cur = S::kSent; break; }
                }
            }
            if (any && best_id >= 0) { leaf = 0; break; }
            leaf = cur;
            if (cur < 0) {
                cur = stk.get(sp);
                sp -= S::kStep;
            }
            // back to the inner phase once at most `leaf_exit` lanes still hold a leaf
            // (they keep it postponed); 0: drain every lane's chain of leaves first
            if (__popcll(__ballot(leaf < 0)) <= (uint32_t)leaf_exit) break;
        }
        if (RES && (cur != S::kSent || leaf < 0) && __popcll(__ballot(true)) < min_lanes) break;
        // watchdog: a traversal revisiting nodes forever (corrupt tree) ends the query and
        // raises the fault flag that the host turns into an error, instead of hanging the GPU
        if (++guard > guard_lim) {
            if (fault) atomicOr(fault, 1);
            cur = S::kSent;
            leaf = 0;
        }
    } while (cur != S::kSent || leaf < 0);
    hit_id = best_id;
    hit_t = best;
    if (RES) {
        tsp->cur = cur; tsp->leaf = leaf; tsp->sp = sp; tsp->best_id = best_id; tsp->best = best;
        return !(cur != S::kSent || leaf < 0);
    }
    return best_id >= 0;
}

// Pixel of work item `item` (slot = tile-major, row, column); xy0 = the item's
// tile origin (x0 << 16 | y0).  Uniform inputs are laundered through SGPR asm so
// the compiler cannot hoist their VALU-derived values out of the persistent loop
// (they would pin VGPRs).
// The kernel's TraceParams in the kernarg segment, through a pointer the compiler cannot follow: every
// field read through it is a scalar load (constant cache) at its use instead of a value held in an
// SGPR across the persistent loop
typedef const __attribute__((address_space(4))) TraceParams KParams;
__device__ __forceinline__ KParams& kernarg() {
    // the kernel's only argument sits at the start of the kernarg segment
    KParams* k = (KParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return *k;
}
// trace_kernel: the LDS-scene variants re-read their launch parameters (C1 one-frame launches -13 %,
// C2 -1.5 % against held values spilled into VGPR lanes); the global-scene variant keeps them (C4 +0.8 %
// with re-reads, profiles/r06/kernarg/)
template <bool RELOAD>
__device__ __forceinline__ auto& params(const TraceParams& P) {
    if constexpr (RELOAD) return kernarg();
    else return P;
}
template <class PT>
__device__ __forceinline__ void pixel_of(const PT& P, uint32_t item, uint32_t chunk_s, uint32_t xy0, int& x,
                                         int& y) {
    int log_tw = P.log_tw, log_tpx = P.log_tpx;
    asm volatile("" : "+s"(log_tw), "+s"(log_tpx));
    uint32_t slot = item - chunk_s * (uint32_t)P.n_slots;
    uint32_t loc = slot & ((1u << log_tpx) - 1u);
    x = (int)(xy0 >> 16) + (int)(loc & ((1u << log_tw) - 1u));
    y = (int)(xy0 & 0xFFFFu) + (int)(loc >> log_tw);
}

// Global sample index (the RNG key's sample) of the launch's chunk-relative sample `chunk_s`:
// frame f = j / frame_spp of a multi-frame launch renders samples f * frame_stride + (j % frame_spp)
// (TraceParams::j0).  Wave-uniform operands: one scalar division per chunk or camera wave.
__device__ __forceinline__ uint32_t global_sample(const TraceParams& P, uint32_t chunk_s) {
    uint32_t j = P.j0 + chunk_s, fs = P.frame_spp, st = P.frame_stride, s0 = (uint32_t)P.s0;
    asm volatile("" : "+s"(fs), "+s"(st), "+s"(s0));
    const uint32_t f = j / fs;
    return s0 + f * st + (j - f * fs);
}

// Camera sample for pixel (x, y) of sample `chunk_s` (main_taichi.py:89-95): RNG key,
// jitter, gen_ray.
__device__ __forceinline__ void camera_ray(const TraceParams& P, int x, int y, uint32_t chunk_s, uint32_t& st, V3& o,
                                           V3& d) {
    int W = P.W;
    float wm1 = P.wm1, hm1 = P.hm1;
    asm volatile("" : "+s"(W), "+s"(wm1), "+s"(hm1));
    st = rng_key(P.seed_lo, P.seed_hi, (uint32_t)y * (uint32_t)W + (uint32_t)x, global_sample(P, chunk_s));
    float r0 = rng_next(st);
    float u = ((float)x + r0) / wm1;
    float r1 = rng_next(st);
    float vv = ((float)y + r1) / hm1;
    if (P.cam_fast) {
        // gen_ray for a pinhole affine camera: the same operations minus
        // those with exactly known results (see TraceParams::cam_fast)
        float c[12], k[6];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            c[i] = P.cam[i];
            asm volatile("" : "+s"(c[i]));
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            k[i] = P.cam_o[i];
            k[3 + i] = P.cam_k[i];
            asm volatile("" : "+s"(k[i]), "+s"(k[3 + i]));
        }
        float sd0 = P.cam[16], sd1 = P.cam[17];
        asm volatile("" : "+s"(sd0), "+s"(sd1));
        float rx = (u - 0.5f) * sd0 / 0.5f, ry = (vv - 0.5f) * sd1 / 0.5f;
        float f[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) f[i] = (((rx * c[4 * i] + ry * c[4 * i + 1]) + k[3 + i]) + c[4 * i + 3]) - k[i];
        float ln = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
        o = v3(k[0], k[1], k[2]);
        d = v3(f[0] / ln, f[1] / ln, f[2] / ln);
    } else {
        float cam[24];
#pragma unroll
        for (int i = 0; i < 20; ++i) {
            cam[i] = P.cam[i];
            asm volatile("" : "+s"(cam[i]));
        }
        gen_ray(cam, u, vv, st, o, d);
    }
}

enum : int { Q_EXT = 0, Q_SHADOW = 1, Q_MISL = 2, Q_MISB = 3 };

// MIS direct-lighting variant (VAR & 256): the reference's unused estimator
// PathTracer.sample_direct_lighting2 and its helpers (core/tracing.py:12-90), restated
// as oracle/prt_oracle.c:direct_mis.  Both strategies' visibility tests are closest-hit
// queries over (1e-5, 9999.9) that must land on an emitter; light_area = 1.0 and the
// BRDF strategy's light pdf uses the light-sampled point's normal, as the reference has it.
constexpr float kTMaxMis = 9999.9f;
constexpr float kPiF = 3.14159265358979323846f;   // np.pi inside a Taichi f32 kernel
__device__ __forceinline__ float dot_or_zero(V3 n, V3 l) { float d = dot(n, l); return 0.0f > d ? 0.0f : d; }
__device__ __forceinline__ float mis_power(float pf, float pg) {
    float f = pf * pf, g = pg * pg;
    return f / (f + g);
}
__device__ __forceinline__ float area_light_pdf(float t_light, V3 dir, V3 light_n) {
    float pdf = 0.0f;
    float l_cos = dot(light_n, neg(dir));
    if (l_cos > 1e-4f) {
        V3 tmp = dir * t_light;
        pdf = dot(tmp, tmp) / (1.0f * l_cos);
    }
    return pdf;
}

template <int STACK, bool STATS, int VAR, bool SCENE_LDS, int WPE>
__global__ __attribute__((amdgpu_flat_work_group_size(kBlock, kBlock), amdgpu_waves_per_eu(WPE)))
void trace_kernel(TraceParams P) {
    // VAR bits: 8 phase-aligned scheduling (see below), 32 spill stack, 64 quantised
    // nodes, 128 suspended traversal tails, 256 MIS direct lighting; the traversal is
    // always the while-while BVH4 (traverse_ww4)
    constexpr bool PHASE = (VAR & 8) != 0;
    constexpr bool SPILL = (VAR & 32) != 0;    // LDS stack of STACK entries + global spill area
    constexpr bool QNODE = (VAR & 64) != 0;    // quantised 64-B BVH4 nodes
    constexpr bool RESUME = (VAR & 128) != 0;  // suspend the traversal tail, resume next iteration
    constexpr bool MIS = (VAR & 256) != 0;     // MIS direct lighting (sample_direct_lighting2) instead of NEE
    constexpr bool FSQ = SCENE_LDS;            // shading sqrt fast path (sqrt_cr)
    // the shading quotients' cheap guards (lambert_div, nee_div): LDS scenes; in the global-scene kernel
    // (L1-bound) they measured +0.3 % at C4 (profiles/r06/guards/ab_c4_global_fastdiv.jsonl)
    constexpr bool FDIV = FSQ;
    extern __shared__ float4 smem[];
    // LDS: the traversal stacks (16-bit entries for LDS-resident scenes), then the scene copy
    using StackT = typename std::conditional<SPILL, SpillStack<STACK>,
                                             typename std::conditional<SCENE_LDS, LdsStack16A, LdsStack>::type>::type;
    constexpr int kStackF4 = STACK * kBlock * (SCENE_LDS ? 2 : 4) / 16;
    StackT stk;
    if constexpr (SCENE_LDS) {
        const int t = threadIdx.x;
        stk.base = (int)(uintptr_t)(LdsShort*)(reinterpret_cast<short*>(smem) + (t & ~63) + 2 * (t & 31) + ((t >> 5) & 1));
    } else {
        stk.l = reinterpret_cast<int*>(smem) + threadIdx.x;
    }
    if constexpr (SPILL) {
        stk.g = P.spill + (size_t)blockIdx.x * kBlock + threadIdx.x;
        stk.gs = gridDim.x * kBlock;
    }
    const float4* g_nodes = P.nodes;
    const float4* g_tris = P.tris;
    const float4* s_nm = P.tri_nm;
    const float4* s_fr = P.tri_frame;
    const float* s_mats = P.mats;
    const float4* s_lv = P.light_v;
    const int* s_loff = P.light_off;
    if (SCENE_LDS) {
        // small scene: copy BVH + triangles, and the shading data (normals, frames,
        // materials, emitters), into LDS once per persistent block
        float4* sn = smem + kStackF4;
        const int n_node4 = P.n_node_f4 / 8;
        float4* st4 = sn + 56 * n_node4;
        float4* snm = st4 + P.n_tri_f4;
        float4* sfr = snm + P.n_tri;
        float4* smt = sfr + 6 * P.n_tri;
        float4* slv = smt + 2 * P.n_mat;
        int* slo = reinterpret_cast<int*>(slv + 4 * P.n_lt);
        // octant copies of the BVH4 (visit_node4 OCT): copy k of node n holds the near / far
        // planes of each axis for the direction signs k = sx | sy << 1 | sz << 2, then the refs
        // with the empty-slot reference rewritten to the 16-bit stack's sentinel
        for (int i = threadIdx.x; i < 56 * n_node4; i += kBlock) {
            const int n = i / 56, r = i - 56 * n, k = r / 7, slot = r - 7 * k;
            const int ax = slot >> 1, sgn = (k >> ax) & 1, far = slot & 1;
            const float4* src = P.nodes + 8 * n;
            float4 v = slot == 6 ? src[6] : src[2 * ax + (sgn ^ far)];
            if (slot == 6) {
                int* rr = reinterpret_cast<int*>(&v);
                for (int c = 0; c < 4; ++c) rr[c] = rr[c] == kSentinel ? LdsStack16::kSent : rr[c];
            }
            // copy k orders the children front to back for its direction signs (visit_node4 OCT):
            // ascending near corner along the octant's diagonal, empty slots last, ties by index
            float key[4];
            {
                const float4 lx = src[0], hx = src[1], ly = src[2], hy = src[3], lz = src[4], hz = src[5];
                const float4 rf = src[6];
                const int rr[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
                // near corner of the box, projected on the octant's diagonal
                const float nxv[4] = {lx.x, lx.y, lx.z, lx.w}, fxv[4] = {hx.x, hx.y, hx.z, hx.w};
                const float nyv[4] = {ly.x, ly.y, ly.z, ly.w}, fyv[4] = {hy.x, hy.y, hy.z, hy.w};
                const float nzv[4] = {lz.x, lz.y, lz.z, lz.w}, fzv[4] = {hz.x, hz.y, hz.z, hz.w};
                for (int c = 0; c < 4; ++c) {
                    key[c] = rr[c] == kSentinel ? INFINITY
                                                : ((k & 1) ? -fxv[c] : nxv[c]) + ((k & 2) ? -fyv[c] : nyv[c]) +
                                                      ((k & 4) ? -fzv[c] : nzv[c]);
                    if (!(key[c] == key[c])) key[c] = INFINITY;   // NaN (degenerate box): a total order
                }
            }
            const float vin[4] = {v.x, v.y, v.z, v.w};
            int rank[4];   // position of child c in the order (a permutation of 0..3)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                rank[c] = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) rank[c] += (key[e] < key[c] || (key[e] == key[c] && e < c)) ? 1 : 0;
            }
            // slot j takes the child of rank j (selects, no dynamically indexed array in scratch)
            float vout[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                vout[j] = rank[0] == j ? vin[0] : rank[1] == j ? vin[1] : rank[2] == j ? vin[2] : vin[3];
            sn[i] = make_float4(vout[0], vout[1], vout[2], vout[3]);
        }
        for (int i = threadIdx.x; i < P.n_tri_f4; i += kBlock) st4[i] = P.tris[i];
        for (int i = threadIdx.x; i < P.n_tri; i += kBlock) snm[i] = P.tri_nm[i];
        for (int i = threadIdx.x; i < 6 * P.n_tri; i += kBlock) sfr[i] = P.tri_frame[i];
        for (int i = threadIdx.x; i < 2 * P.n_mat; i += kBlock) smt[i] = reinterpret_cast<const float4*>(P.mats)[i];
        for (int i = threadIdx.x; i < 4 * P.n_lt; i += kBlock) slv[i] = P.light_v[i];
        for (int i = threadIdx.x; i <= P.n_light; i += kBlock) slo[i] = P.light_off[i];
        __syncthreads();
        g_nodes = sn;
        g_tris = st4;
        s_nm = snm;
        s_fr = sfr;
        s_mats = reinterpret_cast<const float*>(smt);
        s_lv = slv;
        s_loff = slo;
    }
    const int lane = threadIdx.x & 63;
    // diagnostic (P.wave_clock, env PRT_WAVE_CLOCK): each wave's start / end real time and the
    // items it took, kept in memory (not registers: the hot loop's VGPR budget is tight)
    if (P.wave_clock && lane == 0)
        P.wave_clock[3 * ((size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6))] = __builtin_amdgcn_s_memrealtime();

    // wave-uniform work queue [q_next, q_end)
    uint32_t q_next = 0, q_end = 0;
    bool exhausted = false;

    // lane state
    TState tst = {0, 0, 0, -1, 0.0f};
    bool pending = false;   // RESUME: a suspended query (state in tst + the LDS stack)
    int item = -1;
    int bounce = 0, qtype = Q_EXT;
    uint32_t st = 0;
    V3 o = v3(0, 0, 0), d = v3(0, 0, 0), wi = v3(0, 0, 0);
    V3 beta = v3(1, 1, 1), L = v3(0, 0, 0), pend = v3(0, 0, 0);
    // MIS: shading normal, light-sampled point's normal, InvPi * rho * light colour, the
    // BRDF-strategy direction and pdf of the current vertex (pend accumulates direct_li)
    V3 mis_n = v3(0, 0, 0), mis_n2 = v3(0, 0, 0), mis_fl = v3(0, 0, 0), mis_bd = v3(0, 0, 0);
    float mis_bp = 0.0f;
    float tmax = kTMax;
    Counters cn = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t w_inner = 0, w_leaf = 0, l_inner = 0, l_leaf = 0;
    uint32_t chunk_s = 0;   // wave-uniform: sample index (within the launch) of the current chunk
    uint32_t chunk_xy0 = 0; // wave-uniform: origin of the current chunk's tile

    // diagnostic (STATS) wave-level clocks: refill / traversal / shading, iterations, active lanes
    uint64_t c_refill = 0, c_trav = 0, c_shade = 0, n_iter = 0, n_active = 0;
    // STATS, phase-aligned schedule: wave clocks and counts of extension / shadow iterations and the
    // lanes that queried in the shadow ones (diag words 17..21)
    uint64_t c_it_ext = 0, c_it_sh = 0, n_it_ext = 0, n_it_sh = 0, lanes_sh = 0, t_it = 0;
    uint64_t t_a = 0, t_b = 0;
    // PHASE: the wave alternates extension and shadow iterations, so the costly
    // shading code (run after extension queries only) and the refill execute
    // with every busy lane at once instead of every iteration with about half.
    // Lanes whose query kind does not match the wave's phase sit the iteration out.
    bool last_shadow = false;
    while (true) {
        // LDS scenes: launch parameters re-read through the kernarg pointer each iteration (see params)
        auto& Q = params<SCENE_LDS>(P);
        if (STATS) { t_a = __builtin_amdgcn_s_memtime(); t_it = t_a; }
        bool do_shadow = false;
        if (PHASE) {
            do_shadow = !last_shadow && __ballot(item >= 0 && qtype == Q_SHADOW) != 0;
            last_shadow = do_shadow;
        }
        // ---------------------------------------------------------- refill
        // me_idle: this lane's own bit of `idle` (kept as a lane predicate: testing the bit
        // needs the 64-bit mask 1 << lane, which the register allocator spilled to scratch)
        bool me_idle = !do_shadow && item < 0;
        uint64_t idle = __ballot(me_idle);
        for (int round = 0; round < 2 && idle; ++round) {
            uint32_t avail = q_end - q_next;
            if (avail == 0 && !exhausted) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(Q.work, (uint32_t)kChunk);
                base = __builtin_amdgcn_readfirstlane(base);
                if ((uint64_t)base >= Q.n_items) {
                    exhausted = true;
                } else {
                    if constexpr (!SCENE_LDS) {
                        // global scenes: queue chunk c -> (sample c % n, 64-pixel group c / n), so
                        // the chunks in flight hold every sample of a few pixel groups instead of
                        // one sample of the whole frame: their paths start (and first bounce) in a
                        // small part of the scene, and its nodes and triangles stay in L2 (C4
                        // 18.12 -> 17.51 ms).  LDS scenes keep sample-major chunks, whose staged
                        // rays and radiance are read and written in address order (pixel-major
                        // there strides 4 MB per chunk: C2 4.23 -> 4.32 ms; profiles/r02/s5/ab_pm/)
                        const uint32_t n_samp = (uint32_t)(Q.n_items / (uint64_t)Q.n_slots);
                        const uint32_t c = base >> 6;
                        const uint32_t g = c / n_samp;
                        base = (c - g * n_samp) * (uint32_t)Q.n_slots + (g << 6);
                        base = __builtin_amdgcn_readfirstlane(base);
                    }
                    q_next = base;
                    q_end = (uint32_t)min((uint64_t)base + kChunk, Q.n_items);
                    if (Q.wave_clock && lane == 0)
                        Q.wave_clock[3 * ((size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) + 2] += q_end - q_next;
                    // n_slots is a multiple of 64 (tile sizes are powers of two >= 64 px),
                    // so a chunk never straddles two samples: one scalar division per chunk
                    chunk_s = __builtin_amdgcn_readfirstlane(base / (uint32_t)Q.n_slots);
                    // tiles hold >= 64 pixels (powers of two), so the chunk lies in one tile
                    uint32_t tk = (base - chunk_s * (uint32_t)Q.n_slots) >> Q.log_tpx;
                    // uniform index: a scalar load through the constant address space
                    chunk_xy0 = ((const __attribute__((address_space(4))) uint32_t*)(uintptr_t)Q.tile_xy)[tk];
                }
                avail = q_end - q_next;
            }
            if (avail == 0) break;
            uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            uint32_t need = (uint32_t)__popcll(idle);
            uint32_t take = need < avail ? need : avail;
            if (me_idle && rank < take) {
                item = (int)(q_next + rank);
                // start a new sample: main_taichi.py:89-95
                L = v3(0, 0, 0);
                int x, y;
                pixel_of(Q, (uint32_t)item, chunk_s, chunk_xy0, x, y);
                int W = Q.W, H = Q.H;
                asm volatile("" : "+s"(W), "+s"(H));
                bool ok = x < W && y < H;
                if (ok) {
                    // primary rays from camera_kernel (or prt_trace_rays' caller rays): no camera code
                    // in the persistent loop, whose uniform operands would spill SGPRs
                    float4 r = Q.rays[item];
                    d = v3(r.x, r.y, r.z);
                    st = __float_as_uint(r.w);
                    if (Q.ray_o) {
                        // per-ray origins: prt_trace_rays' caller rays, thin-lens / projective cameras
                        const float4 ro = Q.ray_o[item];
                        o = v3(ro.x, ro.y, ro.z);
                    } else {
                        float o0 = Q.cam_o[0], o1 = Q.cam_o[1], o2 = Q.cam_o[2];
                        asm volatile("" : "+s"(o0), "+s"(o1), "+s"(o2));
                        o = v3(o0, o1, o2);
                    }
                }
                if (!ok) {
                    float* out = Q.out + (size_t)item * 3;
                    out[0] = 0.0f; out[1] = 0.0f; out[2] = 0.0f;
                    item = -2;  // served, nothing to trace this iteration
                } else {
                    beta = v3(1, 1, 1);
                    bounce = 0;
                    qtype = Q_EXT;
                    tmax = kTMax;
                }
            }
            q_next += take;
            me_idle = item == -1;
            idle = __ballot(me_idle);
        }
        if (item == -2) item = -1;
        if (__ballot(item >= 0) == 0) {
            if (exhausted && q_next == q_end) break;
            continue;
        }
        if (item < 0) continue;
        if (PHASE && (qtype == Q_SHADOW) != do_shadow) continue;

        // ------------------------------------------------------- one query
        int hid = -1;
        float ht = 0.0f;
        bool hit;
        if (STATS) {
            if (!pending) {
                if (qtype == Q_EXT) cn.ext++; else cn.shadow++;
            }
            // wave-level clocks: the first active lane books the interval
            const bool leader = __builtin_amdgcn_readfirstlane(lane) == lane;
            const uint64_t active = __ballot(true);
            t_b = __builtin_amdgcn_s_memtime();
            if (leader) {
                c_refill += t_b - t_a;
                n_iter++;
                n_active += (uint64_t)__popcll(active);
                if (PHASE && do_shadow) lanes_sh += (uint64_t)__popcll(active);
            }
            t_a = t_b;
        }
        // the leaf-phase entry / exit thresholds (counts of lanes) are tuned for full waves; in
        // the drain, with few lanes left, they would switch phase after every trip
        const int lb = exhausted ? 0 : Q.leaf_break, le = exhausted ? 0 : Q.leaf_exit;
        const uint32_t glim = Q.guard_trips;
        if (STATS && !pending) cn.q0 = cn.nodes;   // node visits at the start of this query
        if (RESUME) {
            if (!pending) tstate_init(tst, stk, tmax);
            // suspending a query only pays while idle lanes can be refilled: once the work
            // queue is exhausted (the launch's drain) the wave keeps traversing instead of
            // going round the loop once per inner/leaf phase
            const int res_min = exhausted ? 0 : Q.resume_min;
            bool done;
            if (PHASE && do_shadow)
                done = traverse_ww4<STATS, 2, StackT, QNODE, true, SCENE_LDS>(g_nodes, g_tris, o, d, kTMin, tmax, true, stk, hid,
                                                                  ht, cn, &tst, res_min, Q.fault, lb, le, glim);
            else if (PHASE)
                done = traverse_ww4<STATS, 1, StackT, QNODE, true, SCENE_LDS>(g_nodes, g_tris, o, d, kTMin, tmax, false, stk, hid,
                                                                  ht, cn, &tst, res_min, Q.fault, lb, le, glim);
            else
                done = traverse_ww4<STATS, 0, StackT, QNODE, true, SCENE_LDS>(g_nodes, g_tris, o, d, kTMin, tmax,
                                                                  qtype == Q_SHADOW, stk, hid, ht, cn, &tst, res_min,
                                                                  Q.fault, lb, le, glim);
            pending = !done;
            if (pending) continue;   // resume next iteration; no shading yet
            hit = hid >= 0;
        } else if (PHASE) {
            if (do_shadow)
                hit = traverse_ww4<STATS, 2, StackT, QNODE, false, SCENE_LDS>(g_nodes, g_tris, o, d, kTMin, tmax, true, stk, hid,
                                                                  ht, cn, nullptr, 0, Q.fault, lb, le, glim);
            else
                hit = traverse_ww4<STATS, 1, StackT, QNODE, false, SCENE_LDS>(g_nodes, g_tris, o, d, kTMin, tmax, false, stk, hid,
                                                                  ht, cn, nullptr, 0, Q.fault, lb, le, glim);
        } else {
            hit = traverse_ww4<STATS, 0, StackT, QNODE, false, SCENE_LDS>(g_nodes, g_tris, o, d, kTMin, tmax, qtype == Q_SHADOW,
                                                              stk, hid, ht, cn, nullptr, 0, Q.fault, lb, le, glim);
        }

        if (STATS) {
            const uint32_t qn = cn.nodes - cn.q0;
            cn.max_q = max(cn.max_q, qn);   // most node visits of one query
            // outlier log (diag words 24..151): the first 16 queries with > 1000 node visits
            if (qn > 1000) {
                const unsigned long long k = atomicAdd(Q.stats + 23, 1ull);
                if (k < 16) {
                    unsigned long long* r = Q.stats + 24 + 8 * k;
                    r[0] = __float_as_uint(o.x); r[1] = __float_as_uint(o.y); r[2] = __float_as_uint(o.z);
                    r[3] = __float_as_uint(d.x); r[4] = __float_as_uint(d.y); r[5] = __float_as_uint(d.z);
                    r[6] = __float_as_uint(tmax); r[7] = ((unsigned long long)qtype << 32) | qn;
                }
            }
        }
        if (Q.n_sph > 0 && !(qtype == Q_SHADOW && hit)) {
            // analytic spheres after the triangles (ids n_tri + k), same rule as the oracle
            float best = hit ? ht : tmax;
            for (int k = 0; k < Q.n_sph; ++k) {
                float root;
                if (sphere_hit(Q.sph[k], o, d, kTMin, best, root)) {
                    best = root;
                    hid = Q.n_tri + k;
                    hit = true;
                    if (qtype == Q_SHADOW) break;
                }
            }
            ht = best;
        }
        if (STATS) {
            const bool leader = __builtin_amdgcn_readfirstlane(lane) == lane;
            t_b = __builtin_amdgcn_s_memtime();
            if (leader) c_trav += t_b - t_a;
            t_a = t_b;
            // wave-level loop trips = max over the participating lanes; lane-level = sum
            uint32_t mi = cn.it_inner, ml = cn.it_leaf;
            for (int off = 32; off > 0; off >>= 1) {
                mi = max(mi, (uint32_t)__shfl_xor((int)mi, off));
                ml = max(ml, (uint32_t)__shfl_xor((int)ml, off));
            }
            if (leader) { w_inner += mi; w_leaf += ml; }
            l_inner += cn.it_inner; l_leaf += cn.it_leaf;
            cn.it_inner = 0; cn.it_leaf = 0;
        }
        // ------------------------------------------------- shade the result
        bool finished = false;
        if (qtype == Q_EXT) {
            if (!hit) {
                finished = true;
            } else {
                V3 p = o + d * ht;                                         // ray.at
                V3 ng;
                int mid;
                if (hid < Q.n_tri) {
                    float4 nm = s_nm[hid];
                    ng = xyz(nm);
                    mid = __float_as_int(nm.w);
                } else {                                                   // sphere: (p - c) / r
                    asm volatile("");   // keep the divisions in this branch (no if-conversion)
                    float4 sc = Q.sph[hid - Q.n_tri];
                    ng = v3((p.x - sc.x) / sc.w, (p.y - sc.y) / sc.w, (p.z - sc.z) / sc.w);
                    mid = Q.sph_mat[hid - Q.n_tri];
                }
                const float* m = s_mats + 8 * mid;
                const bool flip = m[4] == 0.0f && dot(ng, neg(d)) < 0.0f;   // shapes.py:101-102
                const V3 n = flip ? neg(ng) : ng;
                if (m[5] == 2.0f || m[5] == 3.0f) {
                    // specular BSDFs (build-added, config 3; bsdf_taichi.py:52-59, :69-86):
                    // delta distributions, beta *= albedo, no NEE
                    bool front = dot(d, ng) < 0.0f;
                    V3 ns = front ? ng : neg(ng);
                    V3 unit = normalize(d);
                    V3 out;
                    bool absorbed = false;
                    if (m[5] == 2.0f) {
                        out = reflect3(unit, ns);
                        if (m[7] > 0.0f) out = out + random_in_unit_sphere(st) * m[7];
                        absorbed = !(dot(out, ns) > 0.0f);
                    } else {
                        float ratio = front ? 1.0f / m[6] : m[6];
                        float ct = -dot(unit, ns);
                        ct = ct > 1.0f ? 1.0f : ct;
                        float stn = sqrtf(1.0f - ct * ct);
                        bool cannot = ratio * stn > 1.0f;
                        if (cannot || schlick(ct, ratio) > rng_next(st)) out = reflect3(unit, ns);
                        else out = refract3(unit, ns, ratio);
                    }
                    if (absorbed) {
                        finished = true;
                    } else {
                        beta = beta * v3(m[0], m[1], m[2]);
                        o = p;
                        d = normalize(out);
                        ++bounce;
                        if (bounce >= Q.depth) finished = true;
                    }
                } else if (m[3] != 0.0f) {                                 // tracing.py:129-139
                    float d1 = dot(neg(d), n);
                    if (d1 > 0.0f) {
                        V3 lc = v3(Q.dl_r, Q.dl_g, Q.dl_b);
                        L = bounce == 0 ? L + lc * beta : L + (lc * beta) * d1;
                    }
                    finished = true;
                } else {
                    // BSDFLambertian.scatter + frame (bsdf.py:29-34, shapes.py:105-108).
                    // Triangles read rotate_z_to's rows precomputed on the host with the
                    // same f32 arithmetic (per face and side); spheres build them here.
                    float u0 = rng_next(st);
                    float u1 = rng_next(st);
                    V3 l = cosine_hemisphere<FSQ>(u0, u1);
                    const float4* fr = s_fr + ((size_t)(hid < Q.n_tri ? hid : 0) * 2 + (flip ? 1 : 0)) * 3;
                    if (hid < Q.n_tri) {
                        float4 f0 = fr[0], f1 = fr[1], f2 = fr[2];
                        wi = normalize<FSQ>(xyz(f0) * l.x + xyz(f1) * l.y + xyz(f2) * l.z);
                    } else {
                        wi = to_world(n, l);
                    }
                    float pdf = fabsf(dot(n, wi)) * kInvPi;
                    V3 att = v3(m[0], m[1], m[2]);
                    float cw = dot(n, wi);
                    float dz = cw > 0.0f ? cw : 0.0f;
                    // tracing.py:146-148: if any component of att*dz/pdf*InvPi is NaN the
                    // reference recomputes it with pdf = 1e-4.  (a / pdf) * InvPi is NaN
                    // exactly when a / pdf is, so the condition is decided before dividing.
                    V3 ad = v3(att.x * dz, att.y * dz, att.z * dz);
                    V3 adp = lambert_div<FDIV>(ad, pdf, cw, Q.shade_fast);
                    V3 nb = v3(adp.x * kInvPi, adp.y * kInvPi, adp.z * kInvPi);
                    beta = beta * nb;
                    // sample_direct_lighting (tracing.py:92-108)
                    int li = Q.n_light > 1 ? rng_int(st, 0, Q.n_light - 1) : 0;
                    int lo = s_loff[li];
                    int f = rng_int(st, 0, s_loff[li + 1] - lo - 1);
                    float su = sqrt_cr<FSQ>(rng_next(st));
                    float sv = rng_next(st);
                    float a = su * (1.0f - sv);
                    float b = su * sv;
                    const float4* lv = s_lv + (size_t)(lo + f) * 4;
                    float4 L0 = lv[0], L1 = lv[1], L2 = lv[2], LN = lv[3];
                    float c = 1.0f - a - b;
                    V3 p2 = (xyz(L0) * a + xyz(L1) * b) + xyz(L2) * c;
                    V3 n2 = xyz(LN);
                    if constexpr (MIS) {
                        // sample_direct_lighting2: the BRDF strategy's direction is drawn now
                        // (queries draw nothing, so the stream order is the reference's)
                        const float* em = s_mats + 8 * __float_as_int(LN.w);
                        mis_fl = v3(m[0] * kInvPi * em[0], m[1] * kInvPi * em[1], m[2] * kInvPi * em[2]);
                        V3 tl = normalize<FSQ>(p2 - p);
                        float b0 = rng_next(st);
                        float b1 = rng_next(st);
                        V3 bl = cosine_hemisphere<FSQ>(b0, b1);
                        if (hid < Q.n_tri) {
                            float4 f0 = fr[0], f1 = fr[1], f2 = fr[2];
                            mis_bd = normalize<FSQ>(xyz(f0) * bl.x + xyz(f1) * bl.y + xyz(f2) * bl.z);
                        } else {
                            mis_bd = to_world(n, bl);
                        }
                        mis_bp = fabsf(dot(n, mis_bd)) * kInvPi;
                        mis_n = n;
                        mis_n2 = n2;
                        pend = v3(0, 0, 0);
                        o = p;
                        tmax = kTMaxMis;
                        if (dot(tl, n) > 0.0f) {
                            d = tl;
                            qtype = Q_MISL;
                        } else if (mis_bp > 0.0f) {
                            d = mis_bd;
                            qtype = Q_MISB;
                        } else {
                            L = L + beta * pend;
                            ++bounce;
                            if (bounce >= Q.depth) finished = true;
                            d = wi;
                            tmax = kTMax;
                        }
                    } else {
                    V3 w = normalize<FSQ>(p2 - p);
                    float t_at = (p2.x - p.x) / w.x;
                    // w2 = normalize(p - p2) is -w bit for bit (round-to-nearest is sign
                    // symmetric) up to the sign of zero components, so dot(n2, w2) =
                    // -dot(n2, w) except for the sign of a zero result, which the
                    // strict "> 0" test and the uses below cannot see.
                    float dot1 = dot(n, w), dot2 = -dot(n2, w);
                    o = p;
                    if (dot1 > 0.0f && dot2 > 0.0f) {
                        const float* em = s_mats + 8 * __float_as_int(LN.w);
                        V3 dd = p - p2;
                        float sl = dot(dd, dd);
                        V3 rad = nee_div<FDIV>(v3(em[0] * dot1 * dot2, em[1] * dot1 * dot2, em[2] * dot1 * dot2), sl,
                                                 dot1, dot2, Q.shade_fast);
                        pend = beta * rad;
                        d = w;
                        tmax = t_at;
                        qtype = Q_SHADOW;
                    } else {
                        // no NEE term possible: go straight to the next bounce
                        ++bounce;
                        if (bounce >= Q.depth) finished = true;
                        d = wi;
                        tmax = kTMax;
                    }
                    }   // !MIS
                }
            }
        } else if (MIS && qtype == Q_MISL) {
            // light strategy: visible when the closest hit is an emitter
            if (hit) {
                const int mid = hid < Q.n_tri ? __float_as_int(s_nm[hid].w) : Q.sph_mat[hid - Q.n_tri];
                if (s_mats[8 * mid + 3] > 0.0f) {
                    float lp = area_light_pdf(ht, d, mis_n2);
                    float bp = dot_or_zero(mis_n, d) / kPiF;
                    if (lp > 0.0f && bp > 0.0f) {
                        float w = mis_power(lp, bp);
                        float nl = dot_or_zero(d, mis_n);
                        pend = pend + v3(mis_fl.x * w * nl / lp, mis_fl.y * w * nl / lp, mis_fl.z * w * nl / lp);
                    }
                }
            }
            if (mis_bp > 0.0f) {
                d = mis_bd;          // o is still the vertex, tmax kTMaxMis
                qtype = Q_MISB;
            } else {
                L = L + beta * pend;
                ++bounce;
                if (bounce >= Q.depth) finished = true;
                d = wi;
                tmax = kTMax;
                qtype = Q_EXT;
            }
        } else if (MIS && qtype == Q_MISB) {
            // BRDF strategy
            if (hit) {
                const int mid = hid < Q.n_tri ? __float_as_int(s_nm[hid].w) : Q.sph_mat[hid - Q.n_tri];
                if (s_mats[8 * mid + 3] > 0.0f) {
                    float lp = area_light_pdf(ht, d, mis_n2);
                    if (lp > 0.0f) {
                        float w = mis_power(mis_bp, lp);
                        float nl = dot_or_zero(d, mis_n);
                        pend = pend + v3(mis_fl.x * w * nl / mis_bp, mis_fl.y * w * nl / mis_bp,
                                         mis_fl.z * w * nl / mis_bp);
                    }
                }
            }
            L = L + beta * pend;
            ++bounce;
            if (bounce >= Q.depth) finished = true;
            d = wi;
            tmax = kTMax;
            qtype = Q_EXT;
        } else {
            if (!hit) L = L + pend;
            ++bounce;
            if (bounce >= Q.depth) finished = true;
            d = wi;           // o is still the hit point p
            tmax = kTMax;
            qtype = Q_EXT;
        }
        if (finished) {
            float* out = Q.out + (size_t)item * 3;
            out[0] = L.x; out[1] = L.y; out[2] = L.z;
            // failure detection (STATS): samples whose radiance is NaN or infinite
            if (STATS && !(isfinite(L.x) && isfinite(L.y) && isfinite(L.z))) cn.nonfinite++;
            item = -1;
        }
        if (STATS) {
            const bool leader = __builtin_amdgcn_readfirstlane(lane) == lane;
            if (leader) {
                const uint64_t t_end = __builtin_amdgcn_s_memtime();
                c_shade += t_end - t_a;
                if (do_shadow) { c_it_sh += t_end - t_it; n_it_sh++; }
                else { c_it_ext += t_end - t_it; n_it_ext++; }
            }
        }
    }
    if (P.wave_clock && lane == 0)
        P.wave_clock[3 * ((size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) + 1] = __builtin_amdgcn_s_memrealtime();
    if (STATS) {
        uint64_t a = cn.nodes, b = cn.tris, c = cn.ext, e = cn.shadow;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_down(a, off); b += __shfl_down(b, off);
            c += __shfl_down(c, off); e += __shfl_down(e, off);
        }
        uint64_t wv[7] = {c_refill, c_trav, c_shade, n_iter, n_active, w_inner, w_leaf};
        for (int k = 0; k < 7; ++k)
            for (int off = 32; off > 0; off >>= 1) wv[k] += __shfl_down(wv[k], off);
        if (lane == 0) {
            atomicAdd(P.stats + 0, (unsigned long long)a);
            atomicAdd(P.stats + 1, (unsigned long long)b);
            atomicAdd(P.stats + 2, (unsigned long long)c);
            atomicAdd(P.stats + 3, (unsigned long long)e);
            for (int k = 0; k < 7; ++k) atomicAdd(P.stats + 4 + k, (unsigned long long)wv[k]);
        }
        {
            uint64_t ph[5] = {c_it_ext, c_it_sh, n_it_ext, n_it_sh, lanes_sh};
            for (int k = 0; k < 5; ++k)
                for (int off = 32; off > 0; off >>= 1) ph[k] += __shfl_down(ph[k], off);
            if (lane == 0)
                for (int k = 0; k < 5; ++k) atomicAdd(P.stats + 17 + k, (unsigned long long)ph[k]);
        }
        {
            uint32_t m = cn.max_sp;
            for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_down((int)m, off));
            if (lane == 0) atomicMax(P.stats + 13, (unsigned long long)m);
            uint32_t nf = cn.nonfinite;
            for (int off = 32; off > 0; off >>= 1) nf += (uint32_t)__shfl_down((int)nf, off);
            if (lane == 0 && nf) atomicAdd(P.stats + 14, (unsigned long long)nf);
            uint32_t mq = cn.max_q;
            for (int off = 32; off > 0; off >>= 1) mq = max(mq, (uint32_t)__shfl_down((int)mq, off));
            if (lane == 0) atomicMax(P.stats + 16, (unsigned long long)mq);
            uint32_t wt = cn.w_tri;
            for (int off = 32; off > 0; off >>= 1) wt += (uint32_t)__shfl_down((int)wt, off);
            if (lane == 0 && wt) atomicAdd(P.stats + 15, (unsigned long long)wt);
        }
        {
            uint64_t a2 = l_inner, b2 = l_leaf;
            for (int off = 32; off > 0; off >>= 1) { a2 += __shfl_down(a2, off); b2 += __shfl_down(b2, off); }
            if (lane == 0) {
                atomicAdd(P.stats + 11, (unsigned long long)a2);
                atomicAdd(P.stats + 12, (unsigned long long)b2);
            }
        }
    }
}

// Block copy of an LDS-resident scene's BVH4 as 8 octant copies per node (visit_node4 OCT): copy
// k of node n holds the near / far planes of each axis for the direction signs k = sx | sy << 1 |
// sz << 2, then the refs with the empty-slot reference rewritten to the 16-bit stack's sentinel,
// the four children in k's front-to-back order (ascending near corner along the octant's
// diagonal, empty slots last, ties by index).  The same layout as trace_kernel's copy loop.
__device__ __forceinline__ void copy_octant_nodes(float4* __restrict__ sn, const float4* __restrict__ nodes,
                                                  int n_node4) {
    for (int i = threadIdx.x; i < 56 * n_node4; i += kBlock) {
        const int n = i / 56, r = i - 56 * n, k = r / 7, slot = r - 7 * k;
        const int ax = slot >> 1, sgn = (k >> ax) & 1, far = slot & 1;
        const float4* src = nodes + 8 * n;
        float4 v = slot == 6 ? src[6] : src[2 * ax + (sgn ^ far)];
        if (slot == 6) {
            int* rr = reinterpret_cast<int*>(&v);
            for (int c = 0; c < 4; ++c) rr[c] = rr[c] == kSentinel ? LdsStack16::kSent : rr[c];
        }
        float key[4];
        {
            const float4 lx = src[0], hx = src[1], ly = src[2], hy = src[3], lz = src[4], hz = src[5];
            const float4 rf = src[6];
            const int rr[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
            const float nxv[4] = {lx.x, lx.y, lx.z, lx.w}, fxv[4] = {hx.x, hx.y, hx.z, hx.w};
            const float nyv[4] = {ly.x, ly.y, ly.z, ly.w}, fyv[4] = {hy.x, hy.y, hy.z, hy.w};
            const float nzv[4] = {lz.x, lz.y, lz.z, lz.w}, fzv[4] = {hz.x, hz.y, hz.z, hz.w};
            for (int c = 0; c < 4; ++c) {
                key[c] = rr[c] == kSentinel ? INFINITY
                                            : ((k & 1) ? -fxv[c] : nxv[c]) + ((k & 2) ? -fyv[c] : nyv[c]) +
                                                  ((k & 4) ? -fzv[c] : nzv[c]);
                if (!(key[c] == key[c])) key[c] = INFINITY;
            }
        }
        const float vin[4] = {v.x, v.y, v.z, v.w};
        int rank[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            rank[c] = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) rank[c] += (key[e] < key[c] || (key[e] == key[c] && e < c)) ? 1 : 0;
        }
        float vout[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            vout[j] = rank[0] == j ? vin[0] : rank[1] == j ? vin[1] : rank[2] == j ? vin[2] : vin[3];
        sn[i] = make_float4(vout[0], vout[1], vout[2], vout[3]);
    }
}

// Block-pooled shadow queries (LDS-resident scenes, the reference estimator).
//
// trace_kernel's phase-aligned waves alternate an extension iteration (62.5 of 64 lanes query at
// config 2) with a shadow iteration in which only the ~38 lanes that drew an NEE ray query, and
// those shadow iterations took 43 % of the wave time.  Here the four waves of a block run in
// lockstep phases instead:
//   E: every wave refills its idle lanes and runs one closest-hit extension query per busy lane,
//      then shades it; a lane whose NEE sample needs a visibility test writes the shadow ray
//      (o = p, d = w, t_max = t_at_light) to its slot of the block's LDS pool and its thread id
//      to the block's shadow queue;
//   S: (after a barrier) the queue's n rays are traversed by the first ceil(n / 64) waves, 64
//      per wave — whichever wave issued them — and each lane writes the any-hit result to the
//      owner's slot; the other waves are idle (their SIMD slots go to other blocks' waves);
//   R: (after a second barrier) each owner adds its pending NEE radiance if unoccluded and moves
//      on to its next bounce.
// So shadow rays are traversed 64 to a wave instead of ~38, and a lane waits for its shadow
// result without blocking its wave's next extension query.  Before writing a shadow ray, the
// lane tests it against the sampled light triangle itself (one exact Moller-Trumbore test in
// the traversal's arithmetic): the reference's t_at_light bound lets the light occlude itself
// (SURVEY.md §0), and such a ray is answered without a query.  The result of every query is
// unchanged (an any-hit query answers "hit" iff some triangle passes the test, whichever is
// tested first), so images stay bit-identical to trace_kernel's and to the oracle's.
//
// LDS (per 256-thread block): the 16-bit traversal stacks (P.lds_stack entries), the pool (7
// f32 arrays of 256: o.xyz, d.xyz, t_max; t_max carries the result back), the queue (256 u8),
// two parity-alternating control words pairs (queue length, "alive"), then the scene copy:
// octant BVH4 nodes, triangles, light triangles and offsets.  Shading data (normals, frames,
// materials) are read from global memory (L1-resident) to keep seven blocks per CU.
constexpr int kPoolF4 = 7 * kBlock / 4;        // pool SoA: 7 x 256 f32
constexpr int kQueueF4 = 2 * kBlock / 16;      // queue: 2 x 256 u8, by iteration parity
constexpr int kCtlF4 = 3;                      // ctl: 12 words
#ifndef PRT_POOL_S_PRIO
#define PRT_POOL_S_PRIO 2
#endif

// One block barrier per iteration (round 4; round 3's kernel had two: after E and after S, with
// the answers resolved in between).  A lane's S answer is resolved in the NEXT iteration, after
// its next extension traversal (which does not depend on it) and before it shades that hit, so
// the reference's order of additions holds and images stay bit-identical.  A wave with a pending
// shadow ray waits only until the previous S phase's chunks are answered (an LDS counter, normally
// done by then); S waves run beside the other waves' next traversals, and waves without a chunk go
// straight on to their refill (C2 4.049 vs 4.080 ms, C3 at 1024^2 x 32 spp 9.455 vs 9.570 ms per
// launch against the two-barrier kernel, profiles/r04/pool1b/).
// PLAIN: the lean build for scenes without spheres and metal / dielectric materials (P.plain; C1, C2,
// C5): without that code the kernel's loop keeps 17 fewer uniform values in spilled SGPRs and is a
// third shorter
template <bool STATS, int WPE, bool PLAIN>
__global__ __attribute__((amdgpu_flat_work_group_size(kBlock, kBlock), amdgpu_waves_per_eu(WPE)))
void trace_kernel_pool(TraceParams P) {
    constexpr int ctl_f4 = kCtlF4;
    extern __shared__ float4 smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int stack_f4 = P.lds_stack * kBlock * 2 / 16;
    // LdsStack16's entry layout with the stack pointer as an LDS address (round 6: C2 -0.2 %, C3 -0.5 %
    // per launch against the index form, profiles/r06/stack/)
    LdsStack16A stk;
    stk.base = (int)(uintptr_t)(LdsShort*)(reinterpret_cast<short*>(smem) + (tid & ~63) + 2 * (tid & 31) +
                                           ((tid >> 5) & 1));
    using Stk = decltype(stk);
    float* pool = reinterpret_cast<float*>(smem + stack_f4);   // [7][256]
    uint8_t* queue = reinterpret_cast<uint8_t*>(smem + stack_f4 + kPoolF4);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(smem + stack_f4 + kPoolF4 + kQueueF4);
    float4* sn = smem + stack_f4 + kPoolF4 + kQueueF4 + ctl_f4;
    const int n_node4 = P.n_node_f4 / 8;
    float4* st4 = sn + 56 * n_node4;
    float4* slv = st4 + P.n_tri_f4;
    int* slo = reinterpret_cast<int*>(slv + 4 * P.n_lt);
    float4* smt = slv + 4 * P.n_lt + (P.n_light + 4) / 4;   // materials, after the light offsets
    copy_octant_nodes(sn, P.nodes, n_node4);
    for (int i = tid; i < P.n_tri_f4; i += kBlock) st4[i] = P.tris[i];
    for (int i = tid; i < 4 * P.n_lt; i += kBlock) slv[i] = P.light_v[i];
    for (int i = tid; i <= P.n_light; i += kBlock) slo[i] = P.light_off[i];
    for (int i = tid; i < 2 * P.n_mat; i += kBlock) smt[i] = reinterpret_cast<const float4*>(P.mats)[i];
    if (tid < 4 * ctl_f4) ctl[tid] = 0u;
    __syncthreads();
    const float4* g_nodes = sn;
    const float4* g_tris = st4;
    // normals and shading frames come from global memory (L1-resident): with either the LDS copy
    // no longer fits seven blocks per CU at config 2; the materials sit in LDS (C2 -1.3 %, C3
    // -1.8 % against global loads, profiles/r03/s9/)
    const float4* s_nm = P.tri_nm;
    const float4* s_fr = P.tri_frame;
    const float* s_mats = reinterpret_cast<const float*>(smt);

    uint32_t q_next = 0, q_end = 0;
    bool exhausted = false;
    int item = -1;
    int bounce = 0;
    bool my_sh = false;      // this lane waits for the result of its pooled shadow ray
    uint32_t st = 0;
    V3 o = v3(0, 0, 0), d = v3(0, 0, 0), wi = v3(0, 0, 0);
    V3 beta = v3(1, 1, 1), L = v3(0, 0, 0), pend = v3(0, 0, 0);
    Counters cn = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t n_e = 0, n_s = 0, lanes_s = 0, pre_hits = 0;
    // STATS lane table (diag words 160..175, tools/lane_table.py): (wave trips, lane trips) of E inner
    // visits, E triangle tests, S inner visits, S triangle tests, the shading block, the Lambert
    // block, the loop iteration (lanes busy after the refill) and the resolve of shadow answers
    uint64_t lt[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // books a traversal's trip counters into lane-table entries k, k + 1 (inner) and k + 2, k + 3 (leaf)
    auto book_trav = [&](int k) {
        lt[k] += cn.wi; lt[k + 1] += cn.li; lt[k + 2] += cn.wl; lt[k + 3] += cn.ll;
        cn.wi = 0; cn.li = 0; cn.wl = 0; cn.ll = 0;
    };
    auto book = [&](int k) {
        uint32_t w = 0, l = 0;
        wave_tick(w, l);
        lt[k] += w; lt[k + 1] += l;
    };
    uint32_t chunk_s = 0, chunk_xy0 = 0;
    // control words (kCtlF4): queue length [0..2], alive [3..5], chunk claims [6..8], S chunks done
    // [9..11], one triple entry per iteration mod 3 (a slot is reset two iterations after its use)
    uint32_t slot = 0, slot_prev = 0, nch_prev = 0;
    // the queue's buffer (2 x 256 entries) alternates with the iteration's parity: entries enqueued in
    // iteration i are read in i's S phase, and the next enqueue into the
    // same buffer (iteration i + 2) comes after barrier i + 1, which every reader has passed
    uint32_t qpar = 0;
#ifdef PRT_POOL_CLOCKS
    // diagnostic build (tools/pool_clocks.py): wave-level cycles in E, at barrier 1, in S, at barrier 2
    uint64_t ck[6] = {0, 0, 0, 0, 0, 0};
    uint64_t t_c = __builtin_amdgcn_s_memtime();
#define PRT_CLOCK(k) do { const uint64_t t_n = __builtin_amdgcn_s_memtime(); ck[k] += t_n - t_c; t_c = t_n; } while (0)
#else
#define PRT_CLOCK(k) do {} while (0)
#endif
    // work-queue refill of the wave's idle lanes (path regeneration, trace_kernel's refill)
    auto refill = [&](KParams& Q) {
            bool me_idle = item < 0;
            uint64_t idle = __ballot(me_idle);
            for (int round = 0; round < 2 && idle; ++round) {
                uint32_t avail = q_end - q_next;
                if (avail == 0 && !exhausted) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(Q.work, (uint32_t)kChunk);
                    base = __builtin_amdgcn_readfirstlane(base);
                    if ((uint64_t)base >= Q.n_items) {
                        exhausted = true;
                    } else {
                        q_next = base;
                        q_end = (uint32_t)min((uint64_t)base + kChunk, Q.n_items);
                        chunk_s = __builtin_amdgcn_readfirstlane(base / (uint32_t)Q.n_slots);
                        uint32_t tk = (base - chunk_s * (uint32_t)Q.n_slots) >> Q.log_tpx;
                        chunk_xy0 = ((const __attribute__((address_space(4))) uint32_t*)(uintptr_t)Q.tile_xy)[tk];
                    }
                    avail = q_end - q_next;
                }
                if (avail == 0) break;
                uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                uint32_t need = (uint32_t)__popcll(idle);
                uint32_t take = need < avail ? need : avail;
                if (me_idle && rank < take) {
                    item = (int)(q_next + rank);
                    L = v3(0, 0, 0);
                    int x, y;
                    pixel_of(Q, (uint32_t)item, chunk_s, chunk_xy0, x, y);
                    int W = Q.W, H = Q.H;
                    asm volatile("" : "+s"(W), "+s"(H));
                    bool ok = x < W && y < H;
                    if (ok) {
                        // primary rays from camera_kernel (or caller rays): no camera code in the loop —
                        // its uniform operands spilled 36 more SGPRs (C2 4.01 -> 3.91 ms without it)
                        float4 r = Q.rays[item];
                        d = v3(r.x, r.y, r.z);
                        st = __float_as_uint(r.w);
                        if (Q.ray_o) {
                            const float4 ro = Q.ray_o[item];
                            o = v3(ro.x, ro.y, ro.z);
                        } else {
                            float o0 = Q.cam_o[0], o1 = Q.cam_o[1], o2 = Q.cam_o[2];
                            asm volatile("" : "+s"(o0), "+s"(o1), "+s"(o2));
                            o = v3(o0, o1, o2);
                        }
                    }
                    if (!ok) {
                        float* out = Q.out + (size_t)item * 3;
                        out[0] = 0.0f; out[1] = 0.0f; out[2] = 0.0f;
                        item = -2;
                    } else {
                        beta = v3(1, 1, 1);
                        bounce = 0;
                        // the primary ray as this lane's next ray (R takes o from the pool, d from wi)
                        pool[0 * kBlock + tid] = o.x; pool[1 * kBlock + tid] = o.y; pool[2 * kBlock + tid] = o.z;
                        wi = d;
                    }
                }
                q_next += take;
                me_idle = item == -1;
                idle = __ballot(me_idle);
            }
        if (item == -2) item = -1;
    };
    while (true) {
        // the launch parameters are re-read each iteration through the kernarg pointer (scalar loads from
        // the constant cache): kept live across the loop they exceeded the SGPR budget and were spilled
        // into VGPR lanes, reloaded by v_readlane in every refill
        KParams& Q = kernarg();
        // ------------------------------------------------------------------ E phase
        refill(Q);
        PRT_CLOCK(4);
        if (STATS && item >= 0) book(12);
        // (a) extension traversal: every busy lane except one whose pending shadow ray ends its path
        const bool trav = item >= 0 && !(my_sh && bounce + 1 >= Q.depth);
        int hid = -1;
        float ht = 0.0f;
        bool hit = false;
        if (__ballot(trav) != 0) {
            if (STATS && lane == __builtin_amdgcn_readfirstlane(lane)) n_e++;
            if (trav) {
                if (STATS) { cn.ext++; cn.q0 = cn.nodes; }
                hit = traverse_ww4<STATS, 1, Stk, false, false, true>(
                    g_nodes, g_tris, o, d, kTMin, kTMax, false, stk, hid, ht, cn, nullptr, 0, Q.fault,
                    exhausted ? 0 : Q.leaf_break, exhausted ? 0 : Q.leaf_exit, Q.guard_trips);
                if (STATS) { cn.max_q = max(cn.max_q, cn.nodes - cn.q0); book_trav(0); }
                if (!PLAIN && Q.n_sph > 0) {
                    float best = hit ? ht : kTMax;
                    for (int k = 0; k < Q.n_sph; ++k) {
                        float root;
                        if (sphere_hit(Q.sph[k], o, d, kTMin, best, root)) {
                            best = root;
                            hid = Q.n_tri + k;
                            hit = true;
                        }
                    }
                    ht = best;
                }
            }
        }
        PRT_CLOCK(5);
        // (b) the previous S phase's answers (its waves ran it beside this wave's traversal): a wave
        // with a pending shadow ray waits until every chunk of the previous queue has been answered
        if (__ballot(my_sh) != 0) {
            // bounded: a wait that never ends (a logic error) raises the watchdog flag instead of
            // hanging the device: 2^20 sleeps of 64 clocks ~ 30 ms, against a worst case of ~0.1 ms for
            // the answers (an LDS scene is <= 24 KiB: a query visits each of its <= ~100 nodes and
            // <= ~500 triangles at most once, ~10^5 cycles even in a STATS build).  A lane whose answer
            // did not arrive ends with NaN radiance (counted by STATS' non-finite samples), so a tripped
            // wait cannot pass for a valid image even before prt_check_faults reports it.
            bool late = false;
            const uint32_t need = nch_prev;
            for (uint32_t spin = 0;
                 need && __hip_atomic_load(&ctl[9 + slot_prev], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need;
                 ++spin) {
                if (spin >= (1u << 20)) {
                    if (lane == 0) atomicOr(Q.fault, 2);
                    late = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (my_sh) {
                if (STATS) book(14);
                const float r = pool[6 * kBlock + tid];
                if (late) L = v3(__int_as_float(0x7FC00000), __int_as_float(0x7FC00000), __int_as_float(0x7FC00000));
                else if (r == r) L = L + pend;   // not occluded
                my_sh = false;
                ++bounce;
                if (bounce >= Q.depth) {
                    float* out = Q.out + (size_t)item * 3;
                    out[0] = L.x; out[1] = L.y; out[2] = L.z;
                    if (STATS && !(isfinite(L.x) && isfinite(L.y) && isfinite(L.z))) cn.nonfinite++;
                    item = -1;
                }
            }
        }
        // (c) shading of this iteration's extension hits
        if (trav) {
            if (STATS) book(8);
            {
                bool finished = false;
                if (!hit) {
                    finished = true;
                } else {
                    V3 p = o + d * ht;
                    V3 ng;
                    int mid;
                    if (PLAIN || hid < Q.n_tri) {
                        float4 nm = s_nm[hid];
                        ng = xyz(nm);
                        mid = __float_as_int(nm.w);
                    } else {
                        asm volatile("");
                        float4 sc = Q.sph[hid - Q.n_tri];
                        ng = v3((p.x - sc.x) / sc.w, (p.y - sc.y) / sc.w, (p.z - sc.z) / sc.w);
                        mid = Q.sph_mat[hid - Q.n_tri];
                    }
                    const float* m = s_mats + 8 * mid;
                    const bool flip = m[4] == 0.0f && dot(ng, neg(d)) < 0.0f;
                    const V3 n = flip ? neg(ng) : ng;
                    if (!PLAIN && (m[5] == 2.0f || m[5] == 3.0f)) {
                        bool front = dot(d, ng) < 0.0f;
                        V3 ns = front ? ng : neg(ng);
                        V3 unit = normalize(d);
                        V3 out;
                        bool absorbed = false;
                        if (m[5] == 2.0f) {
                            out = reflect3(unit, ns);
                            if (m[7] > 0.0f) out = out + random_in_unit_sphere(st) * m[7];
                            absorbed = !(dot(out, ns) > 0.0f);
                        } else {
                            float ratio = front ? 1.0f / m[6] : m[6];
                            float ct = -dot(unit, ns);
                            ct = ct > 1.0f ? 1.0f : ct;
                            float stn = sqrtf(1.0f - ct * ct);
                            bool cannot = ratio * stn > 1.0f;
                            if (cannot || schlick(ct, ratio) > rng_next(st)) out = reflect3(unit, ns);
                            else out = refract3(unit, ns, ratio);
                        }
                        if (absorbed) {
                            finished = true;
                        } else {
                            beta = beta * v3(m[0], m[1], m[2]);
                            wi = normalize(out);   // next ray (p, wi), taken up in R
                            ++bounce;
                            if (bounce >= Q.depth) finished = true;
                        }
                    } else if (m[3] != 0.0f) {
                        float d1 = dot(neg(d), n);
                        if (d1 > 0.0f) {
                            V3 lc = v3(Q.dl_r, Q.dl_g, Q.dl_b);
                            L = bounce == 0 ? L + lc * beta : L + (lc * beta) * d1;
                        }
                        finished = true;
                    } else {
                        if (STATS) book(10);
                        float u0 = rng_next(st);
                        float u1 = rng_next(st);
                        V3 l = cosine_hemisphere<true>(u0, u1);
                        const float4* fr = s_fr + ((size_t)((PLAIN || hid < Q.n_tri) ? hid : 0) * 2 + (flip ? 1 : 0)) * 3;
                        if (PLAIN || hid < Q.n_tri) {
                            float4 f0 = fr[0], f1 = fr[1], f2 = fr[2];
                            wi = normalize<true>(xyz(f0) * l.x + xyz(f1) * l.y + xyz(f2) * l.z);
                        } else {
                            wi = to_world(n, l);
                        }
                        float pdf = fabsf(dot(n, wi)) * kInvPi;
                        V3 att = v3(m[0], m[1], m[2]);
                        float cw = dot(n, wi);
                        float dz = cw > 0.0f ? cw : 0.0f;
                        V3 ad = v3(att.x * dz, att.y * dz, att.z * dz);
                        V3 adp = lambert_div<true>(ad, pdf, cw, Q.shade_fast);
                        V3 nb = v3(adp.x * kInvPi, adp.y * kInvPi, adp.z * kInvPi);
                        beta = beta * nb;
                        int li = Q.n_light > 1 ? rng_int(st, 0, Q.n_light - 1) : 0;
                        int lo = slo[li];
                        int f = rng_int(st, 0, slo[li + 1] - lo - 1);
                        float su = sqrt_cr<true>(rng_next(st));
                        float sv = rng_next(st);
                        float a = su * (1.0f - sv);
                        float b = su * sv;
                        const float4* lv = slv + (size_t)(lo + f) * 4;
                        float4 L0 = lv[0], L1 = lv[1], L2 = lv[2], LN = lv[3];
                        float c = 1.0f - a - b;
                        V3 p2 = (xyz(L0) * a + xyz(L1) * b) + xyz(L2) * c;
                        V3 n2 = xyz(LN);
                        V3 w = normalize<true>(p2 - p);
                        float t_at = (p2.x - p.x) / w.x;
                        float dot1 = dot(n, w), dot2 = -dot(n2, w);
                        bool queued = false;
                        if (dot1 > 0.0f && dot2 > 0.0f) {
                            if (STATS) cn.shadow++;
                            // the sampled light triangle itself, in the traversal's arithmetic: a hit
                            // in (t_min, t_at_light) answers the any-hit query (occluded)
                            float tl;
                            const V3 lv0 = xyz(L0);
                            const bool self_hit = mt_u(lv0, xyz(L1) - lv0, xyz(L2) - lv0, p, w, kTMin, t_at, 0, -1,
                                                       true, tl);
                            if (STATS) { cn.tris++; pre_hits += self_hit ? 1 : 0; }
                            if (!self_hit) {
                                const float* em = s_mats + 8 * __float_as_int(LN.w);
                                V3 dd = p - p2;
                                float sl = dot(dd, dd);
                                V3 rad = nee_div<true>(v3(em[0] * dot1 * dot2, em[1] * dot1 * dot2, em[2] * dot1 * dot2), sl,
                                                         dot1, dot2, Q.shade_fast);
                                pend = beta * rad;
                                pool[3 * kBlock + tid] = w.x; pool[4 * kBlock + tid] = w.y; pool[5 * kBlock + tid] = w.z;
                                pool[6 * kBlock + tid] = t_at;
                                queued = true;
                            }
                        }
                        if (queued) {
                            my_sh = true;
                        } else {
                            ++bounce;
                            if (bounce >= Q.depth) finished = true;
                        }
                    }
                    // every continuing lane parks its next ray's origin p in its pool slot (the
                    // shadow ray's origin too) and its direction in wi: neither stays live in
                    // registers across the S phase, where the lane may traverse another lane's ray
                    pool[0 * kBlock + tid] = p.x; pool[1 * kBlock + tid] = p.y; pool[2 * kBlock + tid] = p.z;
                }
                if (finished) {
                    float* out = Q.out + (size_t)item * 3;
                    out[0] = L.x; out[1] = L.y; out[2] = L.z;
                    if (STATS && !(isfinite(L.x) && isfinite(L.y) && isfinite(L.z))) cn.nonfinite++;
                    item = -1;
                }
            }
        }
        // enqueue this wave's shadow rays: one LDS atomic per wave, thread ids at the ranks
        {
            const uint64_t m = __ballot(my_sh);
            const uint32_t cnt = (uint32_t)__popcll(m);
            uint32_t base = 0;
            if (cnt) {
                if (lane == __builtin_amdgcn_readfirstlane(lane)) base = atomicAdd(&ctl[slot], cnt);
                base = __builtin_amdgcn_readfirstlane(base);
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (my_sh) queue[qpar * kBlock + base + rank] = (uint8_t)tid;
            }
            // a wave with busy lanes or unclaimed work keeps the block looping
            if ((__ballot(item >= 0) != 0 || !exhausted) && lane == 0) ctl[3 + slot] = 1u;
            // the next iteration's words, last used two iterations ago (every wave has read them since)
            if (tid == 0) {
                const uint32_t ns = slot == 2 ? 0u : slot + 1u;
                ctl[ns] = 0u; ctl[3 + ns] = 0u; ctl[6 + ns] = 0u; ctl[9 + ns] = 0u;
            }
        }
        PRT_CLOCK(0);
        __syncthreads();
        PRT_CLOCK(1);
        // ------------------------------------------------------------------ S phase
        const uint32_t n_q = ctl[slot];
        // the queue's rays in ceil(n / 64) chunks, one to each of the first waves to claim one (<= 4
        // chunks, one claim per wave); the others refill the lanes that finished in E meanwhile,
        // off the critical path
        const uint32_t n_chunks = (n_q + 63u) >> 6;
        uint32_t chunk = 0xFFFFFFFFu;
        if (n_chunks) {
            if (lane == 0) chunk = atomicAdd(&ctl[6 + slot], 1u);
            chunk = __builtin_amdgcn_readfirstlane(chunk);
        }
        if (chunk < n_chunks) {
            // the S waves hold up their whole block at barrier 2: issue priority over other blocks
            __builtin_amdgcn_s_setprio(PRT_POOL_S_PRIO);
            // full 64-ray chunks and one partial (equal-size chunks: C2 +0.5 %, C3 +0.8 %; the
            // arrival-ordered claim with an early refill by the first two waves at barrier 1: C2
            // +1.2 %, C3 +0.9 %; profiles/r03/pool/)
            const uint32_t e0 = chunk * 64u, e1 = min(n_q, e0 + 64u);
            const uint32_t e = e0 + (uint32_t)lane;
            if (STATS && lane == 0) { n_s++; lanes_s += e1 - e0; }
            const bool sq = e < e1;
            int owner = 0;
            V3 so = v3(0, 0, 0), sd = v3(1, 1, 1);
            float stm = 0.0f;
            if (sq) {
                owner = queue[qpar * kBlock + e];
                so = v3(pool[0 * kBlock + owner], pool[1 * kBlock + owner], pool[2 * kBlock + owner]);
                sd = v3(pool[3 * kBlock + owner], pool[4 * kBlock + owner], pool[5 * kBlock + owner]);
                stm = pool[6 * kBlock + owner];
            }
            if (sq) {
                int hid = -1;
                float ht = 0.0f;
                if (STATS) cn.q0 = cn.nodes;
                bool hit = traverse_ww4<STATS, 2, Stk, false, false, true>(
                    g_nodes, g_tris, so, sd, kTMin, stm, true, stk, hid, ht, cn, nullptr, 0, Q.fault,
                    exhausted ? 0 : Q.leaf_break, exhausted ? 0 : Q.leaf_exit, Q.guard_trips);
                if (STATS) { cn.max_q = max(cn.max_q, cn.nodes - cn.q0); book_trav(4); }
                if (!PLAIN && Q.n_sph > 0 && !hit) {
                    for (int k = 0; k < Q.n_sph; ++k) {
                        float root;
                        if (sphere_hit(Q.sph[k], so, sd, kTMin, stm, root)) { hit = true; break; }
                    }
                }
                // the result travels back in the owner's t_max word: NaN = occluded
                pool[6 * kBlock + owner] = hit ? __int_as_float(0x7FC00000) : 0.0f;
            }
            __builtin_amdgcn_s_setprio(0);
            // publish the answers (LDS stores above) before counting the chunk as done
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_fetch_add(&ctl[9 + slot], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        nch_prev = n_chunks;
        PRT_CLOCK(2);
        const bool alive = ctl[3 + slot] != 0u;
        slot_prev = slot;
        slot = slot == 2 ? 0u : slot + 1u;
        qpar ^= 1u;
        // the next extension ray: origin from the pool slot, direction wi (no register keeps the
        // previous ray across the S phase, where the lane may traverse another lane's ray)
        o = v3(pool[0 * kBlock + tid], pool[1 * kBlock + tid], pool[2 * kBlock + tid]);
        d = wi;
        if (!alive) break;
    }
#ifdef PRT_POOL_CLOCKS
    if (lane == 0)
        for (int k = 0; k < 6; ++k) atomicAdd(P.stats + 24 + k, (unsigned long long)ck[k]);
#endif
#undef PRT_CLOCK
    if (STATS) {
        uint64_t a = cn.nodes, b = cn.tris, c = cn.ext, e = cn.shadow;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_down(a, off); b += __shfl_down(b, off);
            c += __shfl_down(c, off); e += __shfl_down(e, off);
        }
        uint64_t ph[5] = {n_e, n_s, lanes_s, pre_hits, 0};
        for (int k = 0; k < 4; ++k)
            for (int off = 32; off > 0; off >>= 1) ph[k] += __shfl_down(ph[k], off);
        if (lane == 0) {
            atomicAdd(P.stats + 0, (unsigned long long)a);
            atomicAdd(P.stats + 1, (unsigned long long)b);
            atomicAdd(P.stats + 2, (unsigned long long)c);
            atomicAdd(P.stats + 3, (unsigned long long)e);
            // diag 17..20 (pool kernel): wave E iterations, wave S iterations, lanes of the S
            // iterations, shadow rays answered by the light-triangle test
            for (int k = 0; k < 4; ++k) atomicAdd(P.stats + 17 + k, (unsigned long long)ph[k]);
        }
        for (int k = 0; k < 16; ++k) {
            uint64_t v = lt[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
            if (lane == 0 && v) atomicAdd(P.stats + 160 + k, (unsigned long long)v);
        }
        uint32_t msp = cn.max_sp, nf = cn.nonfinite, mq = cn.max_q;
        for (int off = 32; off > 0; off >>= 1) {
            msp = max(msp, (uint32_t)__shfl_down((int)msp, off));
            nf += (uint32_t)__shfl_down((int)nf, off);
            mq = max(mq, (uint32_t)__shfl_down((int)mq, off));
        }
        if (lane == 0) {
            atomicMax(P.stats + 13, (unsigned long long)msp);
            if (nf) atomicAdd(P.stats + 14, (unsigned long long)nf);
            atomicMax(P.stats + 16, (unsigned long long)mq);
        }
    }
}

}  // namespace

// variant table: (VAR bits of trace_kernel, LDS-resident scene, min waves per SIMD); see prt_kernels.h
// (bit 512: the block-pooled shadow-query kernel trace_kernel_pool)
#define PRT_VARIANTS(X)                       \
    X(kVarLds, 8, true, 7)                    \
    X(kVarLdsAnyOcc, 8, true, 1)              \
    X(kVarGlobal, 224, false, 6)              \
    X(kVarLdsMis, 256, true, 6)               \
    X(kVarLds6, 8, true, 6)                   \
    X(kVarGlobalMis, 480, false, 6)           \
    X(kVarLdsPool, 512, true, 7)              \
    X(kVarLdsPool6, 512, true, 6)

// spill variants exist with LDS stacks of 4 (tests), 16 and 32 entries; the others with 10/16/32
template <int STACK, bool STATS, int VAR, bool LDS, int WPE>
static hipError_t launch_one(const TraceParams& P, int grid, size_t smem, hipStream_t stream) {
    constexpr bool spill = (VAR & 32) != 0;
    if constexpr ((VAR & 512) != 0) {
        // the pool kernel's LDS stack size is a launch parameter (P.lds_stack): one instantiation,
        // compiled in its own unit (prt_trace_pool.hip, other register-allocation flags)
        if constexpr (STACK == 16) return launch_trace_pool(P, STATS, WPE, grid, smem, stream);
        else return hipErrorInvalidValue;
    } else if constexpr (spill ? (STACK == 4 || STACK == 16 || STACK == 32) : (STACK != 4)) {
        trace_kernel<STACK, STATS, VAR, LDS, WPE><<<grid, kBlock, smem, stream>>>(P);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int STACK, bool STATS>
static hipError_t launch_var(const TraceParams& P, int var, int grid, size_t smem, hipStream_t stream) {
    switch (var) {
#define X(id, bits, lds, wpe) \
        case id: return launch_one<STACK, STATS, bits, lds, wpe>(P, grid, smem, stream);
        PRT_VARIANTS(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

template <int STACK, bool STATS, int VAR, bool LDS, int WPE>
static void occ_one(int* n, size_t smem) {
    constexpr bool spill = (VAR & 32) != 0;
    if constexpr ((VAR & 512) != 0) {
        if constexpr (STACK == 16) *n = trace_occ_pool(STATS, WPE, smem);
    } else if constexpr (spill ? (STACK == 4 || STACK == 16 || STACK == 32) : (STACK != 4))
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(n, trace_kernel<STACK, STATS, VAR, LDS, WPE>, kBlock, smem);
}

template <int STACK, bool STATS>
static int occ_var(int var, size_t smem) {
    int n = 0;
    switch (var) {
#define X(id, bits, lds, wpe) \
        case id: occ_one<STACK, STATS, bits, lds, wpe>(&n, smem); break;
        PRT_VARIANTS(X)
#undef X
        default: break;
    }
    return n;
}

}  // namespace prt
