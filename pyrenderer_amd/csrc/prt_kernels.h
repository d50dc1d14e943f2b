// prt_kernels.h — launch interface of the HIP hot path (internal to libprt).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace prt {

// Everything one trace launch needs, passed by value as the kernel argument.
struct TraceParams {
    const float4* nodes;      // BVH2 (4 float4 per node) or BVH4 (8 float4 per node), prt_internal.h
    const float4* tris;       // BVH order, 3 float4 per triangle: (v0,id) (e1,0) (e2,0)
    const float4* tri_nm;     // original order: (face normal xyz, material id bits)
    const float4* tri_frame;  // original order: rotate_z_to rows (x, z, n) for the face normal and its negation
    const float* mats;        // n_mat x 8: rho.rgb, emit, sided, type, ior, roughness
    const float4* light_v;    // per light triangle: V0, V1, V2, (normal xyz, material id bits)
    const int* light_off;     // n_light + 1 prefix offsets into light triangles
    int n_light;
    float dl_r, dl_g, dl_b;   // directly-hit light colour (core/tracing.py:120)
    float cam[24];            // packed camera (include/prt.h)
    // pinhole camera with an affine matrix (no aperture, last row (0,0,0,1), all finite):
    // the ray origin M (0,0,0,1) and the constant terms rd.z * M[i][2] of gen_ray,
    // evaluated on the host in the kernel's f32 order (camera_taichi.py:47-74)
    int cam_fast;
    int* fault;               // watchdog flag (non-zero: a traversal exceeded guard_trips)
    uint32_t guard_trips;     // traversal phases per query before the watchdog trips (env PRT_GUARD_TRIPS)
    int leaf_break;           // while-while: enter the leaf phase when <= this many descending lanes lack a leaf
    int leaf_exit;            // ... and leave it when <= this many lanes still hold a leaf
    int resume_min;           // resume variants: leave the traversal loop below this many active lanes
    int* spill;               // spill variants: per-lane stack entries beyond the LDS part (stride = grid threads)
    const float4* rays;       // primary rays of this launch from camera_kernel, or null (generated in the refill)
    const float4* ray_o;      // prt_trace_rays: per-item ray origin (rays_kernel), or null (the camera's cam_o)
    float cam_o[3], cam_k[3];
    int W, H;                 // full frame (u = (x + r) / (W - 1))
    float wm1, hm1;           // (float)(W - 1), (float)(H - 1)
    int log_tw, log_tpx;      // log2(tile width), log2(tile pixels): tiles are powers of two, >= 64 px
    const uint32_t* tile_xy;  // per tile of this launch: (x0 << 16) | y0
    int n_slots;              // n_tiles * tw * th
    int s0;                   // first sample index of the render (keys the RNG streams with the frame mapping below)
    // several frames in one launch (prt_render_frames_device): the launch's sample index j (chunk
    // offset j0 + the item's sample within the chunk) is sample j % frame_spp of frame j / frame_spp,
    // whose samples start at frame * frame_stride; global sample = s0 + that.  One frame:
    // frame_spp > every j, so the global sample is s0 + j.
    uint32_t j0, frame_spp, frame_stride;
    int depth;
    uint32_t seed_lo, seed_hi;
    uint64_t n_items;         // n_slots * samples in this chunk
    uint32_t* work;           // device work counter (zeroed before the launch)
    float* out;               // n_items x 3 radiance, item = (s - s0) * n_slots + slot
    unsigned long long* stats;  // 4 counters (nodes, tris, ext queries, shadow queries)
    int n_node_f4, n_tri_f4;  // scene sizes in float4 (LDS-resident variant)
    int n_mat, n_lt;          // materials (8 floats each), emitter triangles
    int n_tri;                // hit ids >= n_tri are spheres
    int n_sph;
    const float4* sph;        // center xyz, radius
    const int* sph_mat;
    unsigned long long* wave_clock;  // diagnostic: per wave (start, end, items) real-time stamps, or null
    // camera_kernel clears, before the trace launch that follows it on the stream: bit 0 the work
    // counter (16 B at `work`), bit 1 the watchdog flag (first chunk of a render only) — instead of
    // two memset launches per frame
    int cam_clears;
    int lds_stack;            // pool kernel: 16-bit LDS traversal stack entries per lane (>= the BVH4's need)
    int plain;                // 1: no spheres and no metal / dielectric material (the pool kernel's lean build)
    int shade_fast;           // 1: every material's rho in [2^-40, 2^40] and every face normal's length in
                              // [0.5, 2] (host-checked): the shading quotients' cheap guards (prt_device.h)
};

// trace kernel variants (selectable at run time through PRT_FLAG_VARIANT).  All run the
// while-while BVH4 traversal (prt_device.h traverse_ww4) and give bit-identical images;
// the measured history of the variants this set replaced is in DESIGN.md §2.
constexpr int kVarLds = 1;         // LDS-resident scene, phase-aligned ext/shadow iterations, >= 7 waves/SIMD
                                   // (72 VGPRs: C2 4.40 -> 4.23 ms against the 6-wave build)
constexpr int kVarLdsAnyOcc = 2;   // ... no occupancy target (LDS scenes too large for 6 blocks per CU)
constexpr int kVarGlobal = 3;      // global scene: quantised 64-B nodes, LDS stack + global spill area,
                                   // suspended traversal tails, >= 6 waves/SIMD
// estimator variants: the reference's unused MIS direct lighting (PRT_FLAG_MIS_NEE)
constexpr int kVarLdsMis = 4;      // LDS scene, mixed schedule, >= 6 waves/SIMD
constexpr int kVarGlobalMis = 5;   // kVarGlobal + MIS
constexpr int kVarLds6 = 6;        // kVarLds built for >= 6 waves/SIMD (80 VGPRs): LDS scenes whose copy
                                   // fits six blocks per CU but not seven
constexpr int kVarLdsPool = 7;     // LDS-resident scene, block-pooled shadow queries (trace_kernel_pool),
                                   // >= 7 waves/SIMD; the LDS stack size is P.lds_stack
constexpr int kVarLdsPool6 = 8;    // kVarLdsPool built for >= 6 waves/SIMD (80 VGPRs)
constexpr int kVarFirst = 1;
constexpr int kVarLast = 8;
// ids 9-14 were the round-5 schedules of trace_kernel_pool that did not become the default (fused,
// packed leaf trips, split arrival; DESIGN.md §9, logs in profiles/r05/{fused,pack,split}/): removed
// in round 6, the C-ABI rejects them as unknown variants
bool variant_pool(int var);
bool variant_mis(int var);
bool variant_uses_lds(int var);
bool variant_spills(int var);
bool variant_quantized(int var);

int stack_variant(int bvh_depth);
size_t trace_smem_bytes(int stack, int var, const TraceParams& P);
// camera rays of a launch: rays = (d, rng state); ray_o = per-ray origins (cameras other than the affine
// pinhole; null otherwise)
hipError_t launch_camera(const TraceParams& P, float4* rays, float4* ray_o, hipStream_t stream);
hipError_t launch_hits(const TraceParams& P, bool quantized, bool any, int stack, const float4* rays, int64_t n,
                       int* hit_id, float* hit_t, hipStream_t stream);
// World.hit_all's shading at the closest hits of launch_hits (prt_hit_all): n x 16 f32
hipError_t launch_hit_shade(const TraceParams& P, const float4* rays, int64_t n, const int* hit_id, const float* hit_t,
                            float* out16, hipStream_t stream);
// prt_trace_rays: caller rays (n x 8 f32) -> P.rays (d, rng state keyed (seed, i, 0)) and P.ray_o
// for n_pad >= n items (the padding repeats ray 0)
hipError_t launch_rays_prep(const TraceParams& P, const float* in8, int64_t n, int64_t n_pad, float4* rays,
                            float4* ray_o, hipStream_t stream);
size_t lds_scene_bytes(const TraceParams& P);  // LDS-resident scene + shading data
hipError_t launch_trace(const TraceParams& P, int stack, int var, int grid, bool stats, hipStream_t stream);
// per-frame sample-order sums of one chunk of launch samples [j0, j0 + n): frames f0 .. f0 + n_frames - 1
// (frame f = launch samples [f spp, (f + 1) spp)) into acc + f pitch (floats, >= 3 n_slots), in one launch
hipError_t launch_reduce(const float* buf, float* acc, int n_slots, int64_t j0, int64_t n, int64_t spp, int64_t f0,
                         int64_t n_frames, int64_t pitch, bool accumulate, hipStream_t stream);
// packed tile slots (tile origins tile_xy) -> [x][y] window of the frame (prt_render, prt_render_multi)
hipError_t launch_scatter(const float* packed, const uint32_t* tile_xy, int n_slots, int log_tw, int log_tpx, int x0,
                          int y0, int w, int h, float* out, hipStream_t stream);
// grouped slots (group g at packed + g group_pitch floats, group_slots slots each) of n_frames frames
// (source frame f at + f src_fpitch, output frame f at out + f dst_fpitch), one launch
hipError_t launch_scatter_frames(const float* packed, const uint32_t* tile_xy, int n_slots, int group_slots,
                                 int64_t group_pitch, int n_frames, int64_t src_fpitch, int64_t dst_fpitch, int log_tw,
                                 int log_tpx, int x0, int y0, int w, int h, float* out, hipStream_t stream);
int trace_blocks_per_cu(int stack, int var, bool stats, size_t smem);
// mismatches of the fast reciprocal sequence against 1 / b over all 2^32 floats, by class of |b|
// (8 counters: zero, denormal, < 2^-40, [2^-40, 2^40], (2^40, 2^126], > 2^126, inf, NaN)
hipError_t launch_rcp_selftest(unsigned long long* d_out, hipStream_t stream);
// the fast sequences' guards over all 2^32 floats (10 counters, prt_kernels.hip guard_selftest_kernel)
hipError_t launch_guard_selftest(unsigned long long* d_out, hipStream_t stream);
// the block-pooled shadow-query kernel (prt_trace_pool.hip): launch / blocks per CU by (stats, waves per EU)
// the pooled kernel's lean instantiation (no sphere or specular code) runs when P.plain is set
hipError_t launch_trace_pool(const TraceParams& P, bool stats, int wpe, int grid, size_t smem, hipStream_t stream);
int trace_occ_pool(bool stats, int wpe, size_t smem);

}  // namespace prt
