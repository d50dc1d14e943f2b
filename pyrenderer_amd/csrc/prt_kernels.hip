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
#pragma clang fp contract(off)

#include "prt_device.h"

namespace prt {

// per-(stack, stats) trace-kernel instantiation sets, compiled in parallel from
// prt_trace_inst.hip (one object each)
#define PRT_INST_LIST(X) X(4, 0) X(4, 1) X(10, 0) X(10, 1) X(16, 0) X(16, 1) X(32, 0) X(32, 1)
#define PRT_DECL_INST(S, T)                                                                              \
    hipError_t launch_trace_##S##_##T(const TraceParams& P, int var, int grid, size_t smem, hipStream_t stream); \
    int trace_occ_##S##_##T(int var, size_t smem);
PRT_INST_LIST(PRT_DECL_INST)
#undef PRT_DECL_INST

namespace {

// Primary rays of one launch, generated with every lane busy (the persistent
// trace kernel would otherwise run this code with the few lanes it refills):
// rays[item] = (d, rng state after the camera draws); for cameras other than the affine pinhole
// (TraceParams::cam_fast: the uniform origin cam_o) also ray_o[item] = the ray's origin.
__global__ __launch_bounds__(kBlock) void camera_kernel(TraceParams P, float4* __restrict__ rays,
                                                        float4* __restrict__ ray_o) {
    uint64_t item = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (P.cam_clears & 1) { P.work[0] = 0u; P.work[1] = 0u; P.work[2] = 0u; P.work[3] = 0u; }
        if (P.cam_clears & 2) *P.fault = 0;
    }
    if (item >= P.n_items) return;
    // n_slots is a multiple of 64 (tiles of >= 64 px), so the 64 items of a wave share one sample
    // index: one scalar division per wave from the wave's first item (SGPR operands), instead of
    // a 64-bit division emulated per lane in VALU
    const uint64_t item0 = (uint64_t)blockIdx.x * kBlock + (uint32_t)(__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
    const uint32_t cs = (uint32_t)(item0 / (uint64_t)P.n_slots);
    uint32_t slot = (uint32_t)item - cs * (uint32_t)P.n_slots;
    uint32_t xy0 = P.tile_xy[slot >> P.log_tpx];
    int x, y;
    pixel_of(P, (uint32_t)item, cs, xy0, x, y);
    if (x >= P.W || y >= P.H) return;
    uint32_t st;
    V3 o, d;
    camera_ray(P, x, y, cs, st, o, d);
    // the primary rays are read once, by the trace kernel: a nontemporal store keeps them from
    // displacing the scene in L2 (C2 +0.2 % per bench step; nontemporal accesses inside the trace
    // kernel were +0.1 % at C2 and -0.3 % at C4, so it keeps plain ones)
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v r4 = {d.x, d.y, d.z, __uint_as_float(st)};
    __builtin_nontemporal_store(r4, reinterpret_cast<f4v*>(rays + item));
    if (ray_o) {
        f4v o4 = {o.x, o.y, o.z, 0.0f};
        __builtin_nontemporal_store(o4, reinterpret_cast<f4v*>(ray_o + item));
    }
}

// World.hit_all for a batch of rays (intersection_taichi.py:238-291): closest (or any)
// hit over the BVH4 (float or quantised nodes) then the spheres, one ray per lane.
// rays: n x (o.xyz, tmin), (d.xyz, tmax).  Used by the hit-level parity tests.
template <bool QN, bool ANY>
__global__ __launch_bounds__(kBlock) void hits_kernel(TraceParams P, const float4* __restrict__ rays, int64_t n,
                                                      int* __restrict__ hit_id, float* __restrict__ hit_t) {
    extern __shared__ float4 smem[];
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    LdsStack stk{reinterpret_cast<int*>(smem) + threadIdx.x};
    if (i >= n) return;
    float4 a = rays[2 * i], b = rays[2 * i + 1];
    V3 o = v3(a.x, a.y, a.z), d = v3(b.x, b.y, b.z);
    Counters cn = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    int hid = -1;
    float ht = 0.0f;
    bool hit = traverse_ww4<false, ANY ? 2 : 1, LdsStack, QN>(P.nodes, P.tris, o, d, a.w, b.w, ANY, stk, hid, ht, cn,
                                                              nullptr, 0, P.fault, 0, 0, P.guard_trips);
    if (P.n_sph > 0 && !(ANY && hit)) {
        float best = hit ? ht : b.w;
        for (int k = 0; k < P.n_sph; ++k) {
            float root;
            if (sphere_hit(P.sph[k], o, d, a.w, best, root)) {
                best = root;
                hid = P.n_tri + k;
                hit = true;
                if (ANY) break;
            }
        }
        ht = best;
    }
    hit_id[i] = hit ? hid : -1;
    hit_t[i] = hit ? ht : 0.0f;
}

// World.hit_all's 8-tuple at the closest hits found by hits_kernel (intersection_taichi.py:238-291,
// Quad.hit / Cube.hit shapes.py:76-110): p = o + t d (ray.at), the face normal flipped toward the
// ray for two-sided BSDFs, emitting_light, bsdf.evaluate(), and the scatter: a cosine-hemisphere
// draw (samplers.py:28-32) rotated into rotate_z_to(normal)'s frame (mat4_taichi.py:44-60),
// pdf = |n.wi| / pi.  The two draws come from the stream keyed (seed, ray index, 0).  Spheres
// (build-added) take their normal (p - c) / r and build the frame here.
// out16 per ray: hit, t, p.xyz, n.xyz, emit, rho.rgb, wi.xyz, pdf (zeros after t on a miss).
__global__ __launch_bounds__(kBlock) void hit_shade_kernel(TraceParams P, const float4* __restrict__ rays, int64_t n,
                                                           const int* __restrict__ hit_id,
                                                           const float* __restrict__ hit_t, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 a = rays[2 * i], b = rays[2 * i + 1];
    const V3 o = v3(a.x, a.y, a.z), d = v3(b.x, b.y, b.z);
    float r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = 0.0f;
    const int hid = hit_id[i];
    r[1] = b.w;   // closest_so_far: t_max on a miss
    if (hid >= 0) {
        const float t = hit_t[i];
        const V3 p = o + d * t;
        V3 ng;
        int mid;
        if (hid < P.n_tri) {
            const float4 nm = P.tri_nm[hid];
            ng = xyz(nm);
            mid = __float_as_int(nm.w);
        } else {
            const float4 sc = P.sph[hid - P.n_tri];
            ng = v3((p.x - sc.x) / sc.w, (p.y - sc.y) / sc.w, (p.z - sc.z) / sc.w);
            mid = P.sph_mat[hid - P.n_tri];
        }
        const float* m = P.mats + 8 * mid;
        const bool flip = m[4] == 0.0f && dot(ng, neg(d)) < 0.0f;
        const V3 nn = flip ? neg(ng) : ng;
        uint32_t st = rng_key(P.seed_lo, P.seed_hi, (uint32_t)i, 0u);
        const float u0 = rng_next(st);
        const float u1 = rng_next(st);
        const V3 l = cosine_hemisphere<false>(u0, u1);
        V3 wi;
        if (hid < P.n_tri) {
            const float4* fr = P.tri_frame + ((size_t)hid * 2 + (flip ? 1 : 0)) * 3;
            wi = normalize(xyz(fr[0]) * l.x + xyz(fr[1]) * l.y + xyz(fr[2]) * l.z);
        } else {
            wi = to_world(nn, l);
        }
        const V3 vals[5] = {p, nn, v3(m[0], m[1], m[2]), wi, v3(0, 0, 0)};
        r[0] = 1.0f;
        r[1] = t;
        r[2] = vals[0].x; r[3] = vals[0].y; r[4] = vals[0].z;
        r[5] = vals[1].x; r[6] = vals[1].y; r[7] = vals[1].z;
        r[8] = m[3] != 0.0f ? 1.0f : 0.0f;
        r[9] = vals[2].x; r[10] = vals[2].y; r[11] = vals[2].z;
        r[12] = vals[3].x; r[13] = vals[3].y; r[14] = vals[3].z;
        r[15] = fabsf(dot(nn, wi)) * kInvPi;
    }
    float4* o4 = reinterpret_cast<float4*>(out + 16 * i);
    o4[0] = make_float4(r[0], r[1], r[2], r[3]);
    o4[1] = make_float4(r[4], r[5], r[6], r[7]);
    o4[2] = make_float4(r[8], r[9], r[10], r[11]);
    o4[3] = make_float4(r[12], r[13], r[14], r[15]);
}

// prt_trace_rays: the caller's rays (o.xyz, -, d.xyz, -) as the trace kernel's primary rays —
// (d, rng state keyed (seed, i, 0)) and the origin (o, 0) per item; items past n repeat ray 0
// (the padding to whole 64-item chunks; their radiance is not returned).
__global__ __launch_bounds__(kBlock) void rays_prep_kernel(TraceParams P, const float* __restrict__ in8, int64_t n,
                                                           int64_t n_pad, float4* __restrict__ rays,
                                                           float4* __restrict__ ray_o) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n_pad) return;
    const float* r = in8 + 8 * (i < n ? i : 0);
    const uint32_t st = rng_key(P.seed_lo, P.seed_hi, (uint32_t)i, 0u);
    rays[i] = make_float4(r[4], r[5], r[6], __uint_as_float(st));
    ray_o[i] = make_float4(r[0], r[1], r[2], 0.0f);
}

// Packed tile slots -> a window [x0, x0+w) x [y0, y0+h) of the frame, indexed [x][y]
// like the reference's pixels.to_numpy() (main_taichi.py:25): out[((x-x0)*h + (y-y0))*3 + c].
// tile_xy = (x0 << 16) | y0 per tile (the trace kernel's tile origins); slots outside the
// window (ragged frame edges, tiles straddling the window) are dropped.  Used by
// prt_render (one window) and prt_render_multi (each rank's gathered tiles into the frame).
// Grouped / multi-frame form (prt_scatter_frames): the slots come in groups of `group_slots`
// (one rank's gather block), group g at packed + g * group_pitch floats; frame f = blockIdx.y reads
// at + f * src_fpitch and writes out + f * dst_fpitch (one launch for every frame of a gather)
__global__ __launch_bounds__(kBlock) void scatter_kernel(const float* __restrict__ packed,
                                                         const uint32_t* __restrict__ tile_xy, int n_slots,
                                                         int group_slots, int64_t group_pitch, int64_t src_fpitch,
                                                         int64_t dst_fpitch, int log_tw, int log_tpx, int x0, int y0,
                                                         int w, int h, float* __restrict__ out) {
    int slot = blockIdx.x * kBlock + threadIdx.x;
    if (slot >= n_slots) return;
    uint32_t xy = tile_xy[slot >> log_tpx];
    int r = slot & ((1 << log_tpx) - 1);
    int x = (int)(xy >> 16) + (r & ((1 << log_tw) - 1)) - x0;
    int y = (int)(xy & 0xFFFFu) + (r >> log_tw) - y0;
    if (x < 0 || y < 0 || x >= w || y >= h) return;
    const int g = slot / group_slots;
    const float* p = packed + (size_t)g * group_pitch + 3 * (size_t)(slot - g * group_slots) +
                     (size_t)blockIdx.y * src_fpitch;
    float* o = out + (size_t)blockIdx.y * dst_fpitch + ((size_t)x * h + y) * 3;
    o[0] = p[0]; o[1] = p[1]; o[2] = p[2];
}

// Sequential per-pixel sum over this chunk's samples, in sample order, onto
// the running sums (bit-identical to acc = acc + L[s] for s = 0..spp-1).  One launch covers every
// frame the chunk touches (blockIdx.y): frame f = f0 + y owns the chunk's launch samples
// [max(j0, f spp), min(j0 + n, (f + 1) spp)), summed into acc + f pitch (pitch >= 3 n_slots floats); a
// frame's first samples start its sums (unless accumulating), later chunks continue them.
__global__ __launch_bounds__(kBlock) void reduce_kernel(const float* __restrict__ buf, float* __restrict__ acc0,
                                                        int n_slots, int64_t j0, int64_t n, int64_t spp, int64_t f0,
                                                        int64_t pitch, int accumulate) {
    int slot = blockIdx.x * kBlock + threadIdx.x;
    if (slot >= n_slots) return;
    const int64_t f = f0 + blockIdx.y;
    const int64_t a = max(j0, f * spp), e = min(j0 + n, (f + 1) * spp);
    const int n_spp = (int)(e - a);
    const int first = (a == f * spp) && !accumulate;
    buf += (size_t)(a - j0) * n_slots * 3;
    float* __restrict__ acc = acc0 + (size_t)f * (size_t)pitch;
    float r = 0.0f, g = 0.0f, b = 0.0f;
    if (!first) { r = acc[3 * (size_t)slot]; g = acc[3 * (size_t)slot + 1]; b = acc[3 * (size_t)slot + 2]; }
    for (int s = 0; s < n_spp; ++s) {
        const float* p = buf + ((size_t)s * n_slots + slot) * 3;
        // per-sample radiance is read once here: nontemporal loads
        r = r + __builtin_nontemporal_load(p); g = g + __builtin_nontemporal_load(p + 1);
        b = b + __builtin_nontemporal_load(p + 2);
    }
    acc[3 * (size_t)slot] = r; acc[3 * (size_t)slot + 1] = g; acc[3 * (size_t)slot + 2] = b;
}

}  // namespace

// LDS stack entries of the trace kernel for a BVH4 needing need = depth + 1 entries
// (collapse_bvh4's bound; scenes needing more than 32 take the spill-stack global variant)
int stack_variant(int depth) { return depth + 1 <= 10 ? 10 : depth + 1 <= 16 ? 16 : 32; }

// LDS-resident scene (prt_device.h trace_kernel): the BVH4 as 8 octant copies of 7 float4 per
// node (n_node_f4 counts the 8 float4 of a global BVH4 node), triangles, shading data
size_t lds_scene_bytes(const TraceParams& P) {
    return 16 * (7 * (size_t)P.n_node_f4 + P.n_tri_f4 + 7 * (size_t)P.n_tri + 2 * (size_t)P.n_mat + 4 * (size_t)P.n_lt) +
           4 * ((size_t)P.n_light + 1);
}

size_t trace_smem_bytes(int stack, int var, const TraceParams& P) {
    if (variant_pool(var)) {
        // trace_kernel_pool: 16-bit stacks of P.lds_stack entries, the shadow pool, queue and control
        // words, then the BVH4 octant copies, triangles and light records (no shading data)
        return (size_t)P.lds_stack * kBlock * sizeof(short) +
               16 * (size_t)(kPoolF4 + kQueueF4 + kCtlF4) +
               16 * (7 * (size_t)P.n_node_f4 + P.n_tri_f4 + 4 * (size_t)P.n_lt + ((size_t)P.n_light + 4) / 4 +
                     2 * (size_t)P.n_mat);
    }
    // traversal stack entries: 16-bit for LDS-resident scenes, 32-bit otherwise
    size_t b = (size_t)stack * kBlock * (variant_uses_lds(var) ? sizeof(short) : sizeof(int));
    if (variant_uses_lds(var)) b += lds_scene_bytes(P);
    return b;
}

hipError_t launch_trace(const TraceParams& P, int stack, int var, int grid, bool stats, hipStream_t stream) {
    size_t smem = trace_smem_bytes(stack, var, P);
    switch (stack) {
        case 4: return stats ? launch_trace_4_1(P, var, grid, smem, stream) : launch_trace_4_0(P, var, grid, smem, stream);
        case 10: return stats ? launch_trace_10_1(P, var, grid, smem, stream) : launch_trace_10_0(P, var, grid, smem, stream);
        case 16: return stats ? launch_trace_16_1(P, var, grid, smem, stream) : launch_trace_16_0(P, var, grid, smem, stream);
        case 32: return stats ? launch_trace_32_1(P, var, grid, smem, stream) : launch_trace_32_0(P, var, grid, smem, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_hits(const TraceParams& P, bool quantized, bool any, int stack, const float4* rays, int64_t n,
                       int* hit_id, float* hit_t, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
    size_t smem = (size_t)stack * kBlock * sizeof(int);
    if (quantized) {
        if (any) hits_kernel<true, true><<<grid, kBlock, smem, stream>>>(P, rays, n, hit_id, hit_t);
        else hits_kernel<true, false><<<grid, kBlock, smem, stream>>>(P, rays, n, hit_id, hit_t);
    } else {
        if (any) hits_kernel<false, true><<<grid, kBlock, smem, stream>>>(P, rays, n, hit_id, hit_t);
        else hits_kernel<false, false><<<grid, kBlock, smem, stream>>>(P, rays, n, hit_id, hit_t);
    }
    return hipGetLastError();
}

hipError_t launch_hit_shade(const TraceParams& P, const float4* rays, int64_t n, const int* hit_id, const float* hit_t,
                            float* out16, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hit_shade_kernel<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, stream>>>(P, rays, n, hit_id, hit_t, out16);
    return hipGetLastError();
}

hipError_t launch_rays_prep(const TraceParams& P, const float* in8, int64_t n, int64_t n_pad, float4* rays,
                            float4* ray_o, hipStream_t stream) {
    if (n_pad <= 0) return hipSuccess;
    rays_prep_kernel<<<(unsigned)((n_pad + kBlock - 1) / kBlock), kBlock, 0, stream>>>(P, in8, n, n_pad, rays, ray_o);
    return hipGetLastError();
}

hipError_t launch_scatter(const float* packed, const uint32_t* tile_xy, int n_slots, int log_tw, int log_tpx, int x0,
                          int y0, int w, int h, float* out, hipStream_t stream) {
    return launch_scatter_frames(packed, tile_xy, n_slots, n_slots, 0, 1, 0, 0, log_tw, log_tpx, x0, y0, w, h, out,
                                 stream);
}

hipError_t launch_scatter_frames(const float* packed, const uint32_t* tile_xy, int n_slots, int group_slots,
                                 int64_t group_pitch, int n_frames, int64_t src_fpitch, int64_t dst_fpitch, int log_tw,
                                 int log_tpx, int x0, int y0, int w, int h, float* out, hipStream_t stream) {
    if (n_slots <= 0 || n_frames <= 0) return hipSuccess;
    if (group_slots <= 0 || n_frames > 65535) return hipErrorInvalidValue;
    dim3 grid((unsigned)((n_slots + kBlock - 1) / kBlock), (unsigned)n_frames);
    scatter_kernel<<<grid, kBlock, 0, stream>>>(packed, tile_xy, n_slots, group_slots, group_pitch, src_fpitch,
                                                dst_fpitch, log_tw, log_tpx, x0, y0, w, h, out);
    return hipGetLastError();
}

hipError_t launch_camera(const TraceParams& P, float4* rays, float4* ray_o, hipStream_t stream) {
    int64_t grid = ((int64_t)P.n_items + kBlock - 1) / kBlock;
    camera_kernel<<<(unsigned)grid, kBlock, 0, stream>>>(P, rays, ray_o);
    return hipGetLastError();
}

namespace {
// rcp_fast_seq against the IEEE division 1 / b for every float b (one 2^32 sweep): mismatches counted
// by the class of |b| (prt_selftest_rcp); both NaN counts as equal
__global__ void rcp_selftest_kernel(unsigned long long* out) {
    const uint64_t n = 1ull << 32;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float b = __uint_as_float((uint32_t)i);
        const float r = rcp_fast_seq(b);
        const float e = 1.0f / b;
        const bool same = __float_as_uint(r) == __float_as_uint(e) || (r != r && e != e);
        if (!same) {
            const float ab = fabsf(b);
            const int cat = b == 0.0f ? 0 : (b != b ? 7 : (isinf(b) ? 6 : (ab < 0x1p-126f ? 1 : (ab < 0x1p-40f ? 2 :
                            (ab <= 0x1p40f ? 3 : (ab <= 0x1p126f ? 4 : 5))))));
            atomicAdd(out + cat, 1ull);
        }
    }
}

// The guards of the fast sequences (prt_selftest_guards): one sweep over all 2^32 floats b counts, for
// rcp_fast_seq against 1.0f / b and sqrt_fast_seq against sqrtf (both NaN = equal):
//   0  rcp mismatches the output-class guard accepts (class(r) normal: rcp_exact) — must be 0
//   1  rcp operands the output-class guard sends to the division
//   2  rcp mismatches in all
//   3  rcp mismatches for normal |b| <= 2^126 (round 5's statement) — must be 0
//   4  sqrt mismatches the guard accepts (b >= 2^-96: sqrt_cr) — must be 0
//   5  sqrt operands the guard sends to sqrtf
//   6  sqrt mismatches in all
//   7  sqrt mismatches for b in [2^-96, FLT_MAX] (round 5's range guard) — must be 0
//   8  sqrt mismatches for +0 and +normal b < 2^-96
//   9  sqrt mismatches for denormal b
__global__ void guard_selftest_kernel(unsigned long long* out) {
    const uint64_t n = 1ull << 32;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t c[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float b = __uint_as_float((uint32_t)i);
        auto same = [](float x, float y) { return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y); };
        const float r = rcp_fast_seq(b);
        const bool rs = same(r, 1.0f / b);
        const bool r_ok = rcp_guard_ok(r);
        c[0] += (!rs && r_ok) ? 1u : 0u;
        c[1] += r_ok ? 0u : 1u;
        c[2] += rs ? 0u : 1u;
        c[3] += (!rs && __builtin_amdgcn_classf(b, kClassNormal) && fabsf(b) <= 0x1p126f) ? 1u : 0u;
        const float q = sqrt_fast_seq(b);
        const bool qs = same(q, sqrtf(b));
        const bool q_ok = sqrt_guard_ok(b);
        c[4] += (!qs && q_ok) ? 1u : 0u;
        c[5] += q_ok ? 0u : 1u;
        c[6] += qs ? 0u : 1u;
        c[7] += (!qs && b >= 0x1p-96f && b <= 0x1.fffffep127f) ? 1u : 0u;
        c[8] += (!qs && b >= 0.0f && b < 0x1p-96f && __builtin_amdgcn_classf(b, kClassPosNormal | kClassPosZero)) ? 1u : 0u;
        c[9] += (!qs && __builtin_amdgcn_classf(b, kClassDenorm)) ? 1u : 0u;
    }
    for (int k = 0; k < 10; ++k)
        if (c[k]) atomicAdd(out + k, (unsigned long long)c[k]);
}
}  // namespace

hipError_t launch_guard_selftest(unsigned long long* d_out, hipStream_t stream) {
    guard_selftest_kernel<<<4096, 256, 0, stream>>>(d_out);
    return hipGetLastError();
}

hipError_t launch_rcp_selftest(unsigned long long* d_out, hipStream_t stream) {
    rcp_selftest_kernel<<<4096, 256, 0, stream>>>(d_out);
    return hipGetLastError();
}

hipError_t launch_reduce(const float* buf, float* acc, int n_slots, int64_t j0, int64_t n, int64_t spp, int64_t f0,
                         int64_t n_frames, int64_t pitch, bool accumulate, hipStream_t stream) {
    if (n_frames <= 0 || n_frames > 65535 || pitch < 3 * (int64_t)n_slots) return hipErrorInvalidValue;
    dim3 grid((unsigned)((n_slots + kBlock - 1) / kBlock), (unsigned)n_frames);
    reduce_kernel<<<grid, kBlock, 0, stream>>>(buf, acc, n_slots, j0, n, spp, f0, pitch, accumulate ? 1 : 0);
    return hipGetLastError();
}

bool variant_mis(int var) {
    switch (var) {
#define X(id, bits, lds, wpe) case id: return (bits & 256) != 0;
        PRT_VARIANTS(X)
#undef X
        default: return false;
    }
}

bool variant_quantized(int var) {
    switch (var) {
#define X(id, bits, lds, wpe) case id: return (bits & 64) != 0;
        PRT_VARIANTS(X)
#undef X
        default: return false;
    }
}

bool variant_spills(int var) {
    switch (var) {
#define X(id, bits, lds, wpe) case id: return (bits & 32) != 0;
        PRT_VARIANTS(X)
#undef X
        default: return false;
    }
}

bool variant_pool(int var) {
    switch (var) {
#define X(id, bits, lds, wpe) case id: return (bits & 512) != 0;
        PRT_VARIANTS(X)
#undef X
        default: return false;
    }
}

bool variant_uses_lds(int var) {
    switch (var) {
#define X(id, bits, lds, wpe) case id: return lds;
        PRT_VARIANTS(X)
#undef X
        default: return false;
    }
}

int trace_blocks_per_cu(int stack, int var, bool stats, size_t smem) {
    switch (stack) {
        case 4: return stats ? trace_occ_4_1(var, smem) : trace_occ_4_0(var, smem);
        case 10: return stats ? trace_occ_10_1(var, smem) : trace_occ_10_0(var, smem);
        case 16: return stats ? trace_occ_16_1(var, smem) : trace_occ_16_0(var, smem);
        case 32: return stats ? trace_occ_32_1(var, smem) : trace_occ_32_0(var, smem);
        default: return 0;
    }
}

}  // namespace prt
