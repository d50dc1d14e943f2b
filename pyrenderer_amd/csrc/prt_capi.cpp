// prt_capi.cpp — the extern "C" surface of libprt (declared in include/prt.h).
//
// Owns device residency of a scene (BVH, triangles, materials, lights), the
// per-call workspaces (chunked per-sample radiance buffer, work counter), and
// the launch sequence: memset(counter) -> trace_kernel -> reduce_kernel per
// sample chunk, all on one stream.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/prt.h"
#include "prt_internal.h"
#include "prt_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(PRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

float bits_f(int32_t v) { float f; std::memcpy(&f, &v, 4); return f; }

// rotate_to / rotate_z_to rows (mathematics/mat4_taichi.py:9-52) for a normal,
// in the kernel's f32 arithmetic (this file is compiled with -ffp-contract=off):
// rows (x, z, v) with v = normalize(n), x = normalize(v x (0,1,0)), z = normalize(x x v).
struct F3 { float x, y, z; };
F3 f3_norm(F3 a) {
    float l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return F3{a.x / l, a.y / l, a.z / l};
}
F3 f3_cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
void frame_rows(F3 n, float* out12) {
    F3 v = f3_norm(n);
    F3 r1, r2, r3;
    if (v.y == 1.0f) {
        r1 = F3{1, 0, 0}; r2 = F3{0, 0, 1}; r3 = F3{0, 1, 0};
    } else if (v.y == -1.0f) {
        r1 = F3{1, 0, 0}; r2 = F3{0, 0, 1}; r3 = F3{0, -1, 0};
    } else {
        F3 x = f3_norm(f3_cross(v, F3{0.0f, 1.0f, 0.0f}));
        F3 z = f3_norm(f3_cross(x, v));
        r1 = x; r2 = z; r3 = v;
    }
    const F3 rows[3] = {r1, r2, r3};
    for (int k = 0; k < 3; ++k) {
        out12[4 * k] = rows[k].x; out12[4 * k + 1] = rows[k].y; out12[4 * k + 2] = rows[k].z; out12[4 * k + 3] = 0.0f;
    }
}

// stats words: nodes, tris, ext, shadow (public) + diagnostic wave clocks
// (refill, traversal, shading), wave iterations, active lanes at traversal; words 24..151 the outlier
// log, 160..175 the pooled kernel's lane table (STATS builds)
constexpr int kStatWords = 192;

// Device buffer owned by its holder: freed by release() or, at the latest, by the destructor (the
// per-call buffers of prt_trace_rays / prt_closest_hits / prt_hit_all are locals, freed on return
// after their stream has been synchronised; round 4 leaked them on every call).  Not copyable.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr; bytes = 0;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; bytes = 0; }
};

// Work buffers of one render stream.  Renders enqueued on distinct streams may run
// concurrently (a frame's tail overlapping the next frame's start), so everything a
// launch writes lives here: tile origins, per-sample radiance and primary rays, the
// work counter + watchdog flag, the spill area and the host-output sums.
struct RenderCtx {
    hipStream_t stream = nullptr;
    DevBuf tiles, buf, rays, rays_o, work, acc, spill;
    std::vector<uint32_t> tile_host;   // tile origins of the last upload (== device copy in `tiles`)
    uint64_t last_use = 0;
};
constexpr size_t kMaxCtx = 8;

struct Scene {
    int device = 0;
    int64_t n_tri = 0;
    int64_t n_nodes = 0;
    int32_t depth = 0;
    int n_light = 0;
    int n_mat = 0;
    int cus = 0;
    int blocks_per_cu = 0;           // of the default variant
    int occ[2 * (prt::kVarLast + 1)] = {0};  // blocks/CU per (variant, stats) once queried
    int n_lt = 0;                    // emitter triangles
    int64_t n_tri_f4 = 0;
    float direct_rgb[3] = {0.9f, 0.85f, 0.7f};
    DevBuf nodes4q;                  // quantised BVH4 (prt_internal.h)
    int64_t n_node4q_f4 = 0;
    DevBuf nodes4, tris, tri_nm, tri_frame, mats, light_v, light_off, sph, sph_mat;
    int64_t n_node4_f4 = 0;
    int32_t depth4 = 0;
    int stack4 = 0;                  // stack variant for the BVH4 (0 = BVH4 unusable)
    int need4 = 0;                   // worst-case BVH4 traversal stack entries
    int leaf_break = -1;             // env PRT_LEAF_BREAK (0..64); -1: per variant (trace launch)
    int leaf_exit = -1;              // env PRT_LEAF_EXIT (0..64); -1: per variant (trace launch)
    int resume_min = 32;             // resume variants (env PRT_RESUME_MIN; C4 after the r02 BVH fixes: 16 / 24 / 32 / 40 / 48 -> 19.4 / 19.1 / 19.0 / 19.4 / 19.8 ms)
    uint32_t guard_trips = 1u << 20; // traversal phases per query before the watchdog trips (env PRT_GUARD_TRIPS)
    int spill_lds = 16;              // LDS part of the spill variants' stack (env PRT_SPILL_LDS: 4, 16 or 32)
    std::string wave_clock_path;     // env PRT_WAVE_CLOCK: append each trace launch's per-wave clocks here
    int64_t n_sph = 0;
    bool plain = false;              // no spheres, no metal / dielectric material (TraceParams::plain)
    bool shade_fast = false;         // TraceParams::shade_fast (prt_scene_create)
    DevBuf work, stats;              // work: hit-query watchdog flag; stats: PRT_FLAG_STATS counters
    hipStream_t stream = nullptr;
    std::vector<std::unique_ptr<RenderCtx>> ctx;  // per render stream (<= kMaxCtx)
    uint64_t use_clock = 0;
    std::vector<hipEvent_t> ev;   // start/stop pairs of the last timed call
    int ev_used = 0;
    // per-sample buffer budget of one trace launch (radiance + primary rays): 16 GiB of the 288 GB
    // of HBM makes config 3 one launch per frame and config 5 eight (4 GiB: 2 and 29), +0.4 / +0.5 %
    // from the launch tails saved (profiles/r02/s5/chunk_ab/)
    size_t chunk_bytes = (size_t)16 << 30;
    size_t device_bytes = 0;
    // prt_render / prt_render_multi (as the root): [x][y] output frame, gathered tile sums
    // of every rank and their tile origins (host copy kept alive for the async upload)
    DevBuf frame, gather, gather_xy;
    std::vector<uint32_t> gather_xy_host;
    // prt_scatter_tiles: tile origins of the last upload (host copy alive until it has run, i.e.
    // until scatter_ev completes; re-uploaded only when a call's tile set differs)
    DevBuf scatter_xy;
    std::vector<uint32_t> scatter_xy_host;
    hipEvent_t scatter_ev = nullptr;
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) { (void)hipGetDevice(&prev); (void)hipSetDevice(dev); }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

int upload(DevBuf& b, const void* host, size_t bytes, size_t* total) {
    HIP_TRY(b.ensure(std::max<size_t>(bytes, 16)));
    if (bytes) HIP_TRY(hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice));
    *total += b.bytes;
    return PRT_OK;
}

void destroy_scene(Scene* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    for (DevBuf* b : {&s->nodes4q, &s->nodes4, &s->tris, &s->tri_nm, &s->tri_frame, &s->mats, &s->light_v,
                      &s->light_off, &s->sph, &s->sph_mat, &s->work, &s->stats, &s->frame, &s->gather,
                      &s->gather_xy, &s->scatter_xy})
        b->release();
    if (!s->ctx.empty()) (void)hipDeviceSynchronize();
    for (auto& c : s->ctx)
        for (DevBuf* b : {&c->tiles, &c->buf, &c->rays, &c->rays_o, &c->work, &c->acc, &c->spill})
            b->release();
    for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
    if (s->scatter_ev) (void)hipEventDestroy(s->scatter_ev);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

int check_render_args(Scene* s, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids,
                      int n_tiles, int spp, int depth) {
    if (!s) return fail(PRT_ERR_ARG, "scene is NULL");
    if (!cam) return fail(PRT_ERR_ARG, "cam is NULL");
    if (W < 2 || H < 2) return fail(PRT_ERR_ARG, "W and H must be >= 2 (u = (x + r) / (W - 1))");
    if (tw < 1 || th < 1 || (tw & (tw - 1)) || (th & (th - 1)) || (int64_t)tw * th < 64 || (int64_t)tw * th > (1 << 20))
        return fail(PRT_ERR_ARG, "tile width/height must be powers of two with 64 <= tw*th <= 2^20");
    if (W > 65535 || H > 65535) return fail(PRT_ERR_ARG, "frame larger than 65535 pixels per side");
    if (n_tiles < 0 || (n_tiles > 0 && !tile_ids)) return fail(PRT_ERR_ARG, "bad tile list");
    if (spp < 0 || depth < 0) return fail(PRT_ERR_ARG, "spp and depth must be >= 0");
    int tiles_x = (W + tw - 1) / tw, tiles_y = (H + th - 1) / th;
    for (int i = 0; i < n_tiles; ++i)
        if (tile_ids[i] < 0 || tile_ids[i] >= tiles_x * tiles_y)
            return fail(PRT_ERR_ARG, "tile id out of range: " + std::to_string(tile_ids[i]));
    if ((int64_t)n_tiles * tw * th >= ((int64_t)1 << 31)) return fail(PRT_ERR_ARG, "too many pixels in one call");
    return PRT_OK;
}

// work.p: [0] chunk counter; [kFaultOffset] traversal watchdog flag
constexpr size_t kFaultOffset = 32;

// Reads a watchdog flag and clears it once read, so every fault is reported exactly once:
// by the call whose launch raised it (host-output renders, hit queries), or by the first
// prt_check_faults / prt_kernel_timing after a device-output render.  A flag left set would
// otherwise be reported against every later, clean render (callers synchronise first).
int take_fault_at(const DevBuf& work) {
    int f = 0;
    if (!work.p) return 0;
    if (hipMemcpy(&f, (char*)work.p + kFaultOffset, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (f != 0 && hipMemset((char*)work.p + kFaultOffset, 0, sizeof(int)) != hipSuccess) return -1;
    return f;
}
int take_fault(Scene* s) { return take_fault_at(s->work); }
// every render context's watchdog flag (all are taken, not only the first one set)
int take_render_faults(Scene* s) {
    int any = 0;
    for (auto& c : s->ctx)
        if (int f = take_fault_at(c->work)) any = any ? any : f;
    return any;
}

// The render context of `stream`, created on first use.  Beyond kMaxCtx streams the
// least recently used context is recycled after a device synchronisation.
RenderCtx* ctx_for(Scene* s, hipStream_t stream) {
    ++s->use_clock;
    for (auto& c : s->ctx)
        if (c->stream == stream) { c->last_use = s->use_clock; return c.get(); }
    if (s->ctx.size() >= kMaxCtx) {
        auto it = std::min_element(s->ctx.begin(), s->ctx.end(),
                                   [](const std::unique_ptr<RenderCtx>& a, const std::unique_ptr<RenderCtx>& b) {
                                       return a->last_use < b->last_use;
                                   });
        if (hipDeviceSynchronize() != hipSuccess) return nullptr;
        (*it)->stream = stream;
        (*it)->last_use = s->use_clock;
        return it->get();
    }
    auto c = std::unique_ptr<RenderCtx>(new (std::nothrow) RenderCtx());
    if (!c) return nullptr;
    if (c->work.ensure(64) != hipSuccess) return nullptr;
    if (hipMemset(c->work.p, 0, 64) != hipSuccess) return nullptr;
    c->stream = stream;
    c->last_use = s->use_clock;
    s->ctx.push_back(std::move(c));
    return s->ctx.back().get();
}

// LDS-resident scene: BVH + triangles small enough to sit beside the stack
constexpr int64_t kLdsSceneBytes = 24 * 1024;
void scene_sizes(const Scene* s, prt::TraceParams& P) {
    P.n_node_f4 = (int)s->n_node4_f4;
    P.n_tri_f4 = (int)s->n_tri_f4;
    P.n_tri = (int)s->n_tri;
    P.n_mat = s->n_mat;
    P.n_lt = s->n_lt;
    P.n_light = s->n_light;
}
// ... and whose node indices and leaf references fit the LDS kernels' 16-bit stack entries
// (inner nodes < 0x7FFF, the sentinel; leaf refs >= -32768)
bool lds_fits4(const Scene* s) {
    prt::TraceParams P;
    std::memset(&P, 0, sizeof(P));
    scene_sizes(s, P);
    const int64_t n_refs = s->n_tri_f4 / 3;
    return (int64_t)prt::lds_scene_bytes(P) <= kLdsSceneBytes && s->n_node4_f4 / 8 < 0x7FFF && n_refs * 8 <= 32768;
}
// LDS-resident scene when it fits; the >= 7 (>= 6) waves/SIMD build when seven (six) blocks'
// LDS still fit one CU (160 KiB), so the occupancy target is not defeated by LDS.
// Everything else (and BVH4s deeper than the 64-entry LDS stack) takes the global-scene
// kernel: 64-B quantised nodes, 16-entry LDS stack + spill, suspended traversal tails,
// >= 6 waves/SIMD (C4: 28.6 ms at 5 waves, 27.2 at 6, 28.6 at 7 with spills).
// An LDS-resident scene whose pooled-shadow kernel still fits seven blocks per CU takes that kernel
// (C2 4.06 vs 4.28 ms, C3 73.6 vs 77.5 ms, profiles/r03/pool/) at every launch size.  Until the
// kernarg re-reads (round 6) launches of fewer than eight items per resident lane kept the
// phase-aligned kernel (round 3: config 1's 65 k items 0.1155 vs 0.1224 ms); with both kernels' spills
// gone the pooled one wins there too: config 1 0.080 vs 0.094 ms per launch, config 2 at 1 / 2 / 4 spp
// 0.245 / 0.351 / 0.490 vs 0.265 / 0.383 / 0.547 ms, the slowest of 8 single-frame shards 0.752 vs
// 0.826 ms (3 frames in flight: 0.634 vs 0.656), profiles/r06/kernarg/variants/.
int default_variant(const Scene* s, int64_t n_items = INT64_MAX) {
    (void)n_items;
    if (!lds_fits4(s) || !s->stack4) return prt::kVarGlobal;
    prt::TraceParams P;
    std::memset(&P, 0, sizeof(P));
    scene_sizes(s, P);
    P.lds_stack = s->need4;
    if (s->need4 <= 32 && prt::trace_smem_bytes(16, prt::kVarLdsPool, P) * 7 <= 160 * 1024)
        return prt::kVarLdsPool;
    size_t smem = prt::trace_smem_bytes(s->stack4, prt::kVarLds, P);
    return smem * 7 <= 160 * 1024 ? prt::kVarLds : smem * 6 <= 160 * 1024 ? prt::kVarLds6 : prt::kVarLdsAnyOcc;
}
// the traversal stack entries of variant `var` (LDS part for the spill variants; the pool kernel's
// instantiation set, its LDS stack being the launch parameter P.lds_stack)
int variant_stack(const Scene* s, int var) {
    return prt::variant_pool(var) ? 16 : prt::variant_spills(var) ? s->spill_lds : s->stack4;
}

// Pinhole camera with an affine matrix (no aperture, last row (0,0,0,1), all finite):
// the kernels may use the exact gen_ray shortcut (TraceParams::cam_fast).
bool camera_is_fast(const float* cam) {
    bool fin = true;
    for (int i = 0; i < 20; ++i) fin = fin && std::isfinite(cam[i]);
    return fin && !(cam[19] > 0.0f) && cam[12] == 0.0f && cam[13] == 0.0f && cam[14] == 0.0f && cam[15] == 1.0f;
}

// Scene part of a trace launch's parameters (everything but the work description).
void scene_params(Scene* s, prt::TraceParams& P) {
    std::memset(&P, 0, sizeof(P));
    P.nodes = (const float4*)s->nodes4.p;
    P.tris = (const float4*)s->tris.p;
    P.tri_nm = (const float4*)s->tri_nm.p;
    P.tri_frame = (const float4*)s->tri_frame.p;
    P.mats = (const float*)s->mats.p;
    P.light_v = (const float4*)s->light_v.p;
    P.light_off = (const int*)s->light_off.p;
    P.n_light = s->n_light;
    P.dl_r = s->direct_rgb[0]; P.dl_g = s->direct_rgb[1]; P.dl_b = s->direct_rgb[2];
    P.resume_min = s->resume_min;
    P.stats = (unsigned long long*)s->stats.p;
    scene_sizes(s, P);
    P.guard_trips = s->guard_trips;
    P.n_sph = (int)s->n_sph;
    P.sph = (const float4*)s->sph.p;
    P.sph_mat = (const int*)s->sph_mat.p;
    P.plain = s->plain ? 1 : 0;
    P.shade_fast = s->shade_fast ? 1 : 0;
    P.frame_spp = 0xFFFFFFFFu;   // one frame: global sample = s0 + j0 + the chunk's sample
}

// Kernel variant (flags or the scene's default), its traversal stack, the blocks per CU of
// the persistent grid and the spill area of the global variants; switches P to the quantised
// nodes for the variants that read them.
// the variant a launch of n_items work items takes when the flags name none
int launch_variant(const Scene* s, uint32_t flags, int64_t n_items) {
    int var = (int)((flags >> PRT_FLAG_VARIANT_SHIFT) & 0xFFu);
    const bool mis = (flags & PRT_FLAG_MIS_NEE) != 0;
    if (var == 0)
        var = !mis ? default_variant(s, n_items) : (lds_fits4(s) && s->stack4) ? prt::kVarLdsMis : prt::kVarGlobalMis;
    return var;
}

int trace_setup(Scene* s, RenderCtx* cx, uint32_t flags, int64_t n_items, prt::TraceParams& P, int* var_out,
                int* stack_out, int* occ_out) {
    const bool stats = (flags & PRT_FLAG_STATS) != 0;
    const bool mis = (flags & PRT_FLAG_MIS_NEE) != 0;
    int var = launch_variant(s, flags, n_items);
    if (var < prt::kVarFirst || var > prt::kVarLast) return fail(PRT_ERR_ARG, "unknown kernel variant");
    if (prt::variant_mis(var) != mis)
        return fail(PRT_ERR_ARG, "PRT_FLAG_MIS_NEE must be set exactly for the MIS estimator variants");
    const bool spill = prt::variant_spills(var);
    if (s->stack4 == 0 && !spill) return fail(PRT_ERR_ARG, "BVH4 too deep for the LDS traversal stack variants");
    const int stack = variant_stack(s, var);
    if (prt::variant_quantized(var)) {
        P.nodes = (const float4*)s->nodes4q.p;
        P.n_node_f4 = (int)s->n_node4q_f4;
    }
    if (prt::variant_uses_lds(var) && !lds_fits4(s)) return fail(PRT_ERR_ARG, "scene too large for the LDS variant");
    if (prt::variant_pool(var) && (s->need4 > 32 || s->need4 < 1))
        return fail(PRT_ERR_ARG, "BVH4 too deep for the pooled-shadow variant's LDS stack");
    // while-while leaf-phase entry: LDS scenes wait for every descending lane's leaf (their
    // leaves are cheap and traversals short); global scenes enter the leaf phase once at
    // most 16 descending lanes still lack one (C4: 35.1 -> 29.7 ms at 8 in round 1, 18.69 ->
    // 18.44 ms at 16 with leaf exit 12 after the round-2 traversal changes; C2 prefers 0).
    // Leaf-phase exit: back to descending once at most 8 (LDS) / 24 (global) lanes still
    // hold a leaf (C2 5.25 -> 5.04 ms in round 1, flat for 8-16 now; C4 with pixel-major
    // chunks 17.37-17.46 ms at 24 against 17.50-17.64 at 12 in three interleaved rounds,
    // profiles/r03/s1_baseline/leafexit/)
    const bool lds_var = prt::variant_uses_lds(var);
    P.lds_stack = s->need4;
    P.leaf_break = s->leaf_break >= 0 ? s->leaf_break : (lds_var ? 0 : 16);
    P.leaf_exit = s->leaf_exit >= 0 ? s->leaf_exit : (lds_var ? 8 : 24);
    int& occ = s->occ[2 * var + (stats ? 1 : 0)];
    if (occ == 0) occ = std::max(1, prt::trace_blocks_per_cu(stack, var, stats, prt::trace_smem_bytes(stack, var, P)));
    if (spill) {
        // entries [spill_lds, need4] of every lane of the largest grid, plus one slot of headroom
        size_t per_lane = (size_t)std::max(1, s->need4 + 2 - s->spill_lds);
        HIP_TRY(cx->spill.ensure(per_lane * (size_t)occ * s->cus * 256 * sizeof(int)));
        P.spill = (int*)cx->spill.p;
    }
    *var_out = var;
    *stack_out = stack;
    *occ_out = occ;
    return PRT_OK;
}

// Camera and frame part of a launch's parameters (camera_kernel's gen_ray inputs): the record, the
// pinhole shortcut's host-evaluated constant terms (TraceParams::cam_fast), resolution and tiling.
void camera_params(prt::TraceParams& P, const float* cam, int W, int H, int tw, int th) {
    std::memcpy(P.cam, cam, sizeof(float) * PRT_CAM_FLOATS);
    P.cam_fast = camera_is_fast(cam) ? 1 : 0;
    const float rd2 = -cam[18];
    for (int i = 0; i < 3; ++i) {
        const float* c = cam + 4 * i;
        P.cam_o[i] = 0.0f * c[0] + 0.0f * c[1] + 0.0f * c[2] + 1.0f * c[3];
        P.cam_k[i] = rd2 * c[2];
    }
    P.W = W; P.H = H;
    P.wm1 = (float)(W - 1); P.hm1 = (float)(H - 1);
    P.log_tw = __builtin_ctz((unsigned)tw);
    P.log_tpx = __builtin_ctz((unsigned)(tw * th));
}

// Enqueue the whole render of a tile set on `stream`, result in d_acc: samples
// first_sample .. first_sample + spp - 1 of every pixel; `accumulate` adds them onto the
// sums already in d_acc (progressive rendering) instead of overwriting them.
// n_frames > 1 (prt_render_frames_device): frame f renders samples first_sample + f * frame_stride
// + 0 .. spp - 1 into d_acc + f * out_pitch floats (0: packed, n_slots * 3), and all frames' items run
// through the same
// persistent launches (a launch covers up to the memory budget's worth of frames), so the
// launch drains once per launch instead of once per frame.
int enqueue_render(Scene* s, RenderCtx* cx, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids,
                   int n_tiles, int spp, int depth, uint64_t seed, uint32_t flags, float* d_acc,
                   int first_sample = 0, bool accumulate = false, int n_frames = 1, int frame_stride = 0,
                   int64_t out_pitch = 0) {
    if (flags & PRT_FLAG_NO_PRIMARY_KERNEL)
        return fail(PRT_ERR_UNSUP, "PRT_FLAG_NO_PRIMARY_KERNEL: camera rays always come from the camera kernel "
                                   "(the trace kernels no longer carry camera code)");
    const int64_t n_slots = (int64_t)n_tiles * tw * th;
    if (n_slots == 0) return PRT_OK;
    if (out_pitch == 0) out_pitch = 3 * n_slots;
    hipStream_t stream = cx->stream;
    // per-tile pixel origins (x0 << 16 | y0); uploaded only when they differ from the
    // context's last upload (a bench or animation re-renders the same tile set every
    // frame), so a steady-state frame enqueues no host-to-device copy
    const int tiles_x = (W + tw - 1) / tw;
    std::vector<uint32_t> origins((size_t)n_tiles);
    for (int i = 0; i < n_tiles; ++i)
        origins[(size_t)i] = ((uint32_t)((tile_ids[i] % tiles_x) * tw) << 16) | (uint32_t)((tile_ids[i] / tiles_x) * th);
    if (origins != cx->tile_host) {
        HIP_TRY(cx->tiles.ensure(sizeof(uint32_t) * (size_t)n_tiles));
        // the source storage moves into cx->tile_host below and lives until the next upload
        HIP_TRY(hipMemcpyAsync(cx->tiles.p, origins.data(), sizeof(uint32_t) * (size_t)n_tiles, hipMemcpyHostToDevice,
                               stream));
        cx->tile_host.swap(origins);
    }
    if (spp == 0 || depth == 0) {
        // every sample's radiance is 0: the sums are 0, or unchanged when accumulating
        if (!accumulate)
            HIP_TRY(hipMemset2DAsync(d_acc, sizeof(float) * (size_t)out_pitch, 0, sizeof(float) * 3 * (size_t)n_slots,
                                     (size_t)n_frames, stream));
        return PRT_OK;
    }
    // the launches' sample space: j = f * spp + (sample of frame f), T of them
    const int64_t T = (int64_t)spp * n_frames;
    // per-sample buffers: radiance (12 B) + primary ray (16 B) + its origin (16 B, cameras other than
    // the affine pinhole, whose origin is uniform)
    const bool cam_fast = camera_is_fast(cam);
    int64_t per_sample = n_slots * 3 * (int64_t)sizeof(float);
    int64_t per_sample_all = per_sample + n_slots * (cam_fast ? 16 : 32);
    // per-launch budget: the scene's (<= 16 GiB), and when this context's buffers must grow, at
    // most half of the device memory free now plus what they already hold — every render stream
    // (up to kMaxCtx) owns such a buffer set, so a budget fixed at scene creation could ask
    // several streams' worth of the memory that was free then
    size_t budget = s->chunk_bytes;
    {
        const size_t held = cx->buf.bytes + cx->rays.bytes + cx->rays_o.bytes;
        size_t free_b = 0, total_b = 0;
        if ((size_t)(std::min<int64_t>(T, (int64_t)(budget / (size_t)per_sample_all)) * per_sample_all) > held &&
            hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
            budget = std::min(budget, std::max<size_t>((size_t)per_sample_all, (free_b + held) / 2));
    }
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(T, (int64_t)budget / per_sample_all));
    // keep every chunk's item count below 2^31 (32-bit work counter)
    chunk = std::min<int64_t>(chunk, std::max<int64_t>(1, ((int64_t)1 << 31) / n_slots - 1));
    // equal launches: no short last launch paying a whole launch tail for a few samples
    {
        const int64_t nc = (T + chunk - 1) / chunk;
        chunk = (T + nc - 1) / nc;
    }
    HIP_TRY(cx->buf.ensure((size_t)(chunk * per_sample)));
    HIP_TRY(cx->rays.ensure((size_t)(chunk * n_slots * 16)));
    if (!cam_fast) HIP_TRY(cx->rays_o.ensure((size_t)(chunk * n_slots * 16)));
    const bool stats = (flags & PRT_FLAG_STATS) != 0;
    const bool timed = (flags & PRT_FLAG_TIME) != 0;
    if (stats) HIP_TRY(hipMemsetAsync(s->stats.p, 0, kStatWords * sizeof(unsigned long long), stream));

    prt::TraceParams P;
    scene_params(s, P);
    camera_params(P, cam, W, H, tw, th);
    P.rays = (const float4*)cx->rays.p;
    P.ray_o = cam_fast ? nullptr : (const float4*)cx->rays_o.p;
    P.tile_xy = (const uint32_t*)cx->tiles.p;
    P.n_slots = (int)n_slots;
    P.depth = depth;
    P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
    P.work = (uint32_t*)cx->work.p;
    P.fault = (int*)((char*)cx->work.p + kFaultOffset);
    P.out = (float*)cx->buf.p;
    P.s0 = first_sample;
    P.frame_spp = (uint32_t)spp;
    P.frame_stride = (uint32_t)frame_stride;
    int var = 0, stack = 0, occ = 0;
    if (int rc = trace_setup(s, cx, flags, chunk * n_slots, P, &var, &stack, &occ)) return rc;
    int64_t n_chunks = (T + chunk - 1) / chunk;
    // timed launches accumulate event pairs until prt_kernel_timing() reads them
    int k = s->ev_used / 2;
    if (timed) {
        while ((int64_t)s->ev.size() < s->ev_used + 2 * n_chunks) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            s->ev.push_back(e);
        }
        s->ev_used += (int)(2 * n_chunks);
    }
    for (int64_t s0 = 0; s0 < T; s0 += chunk, ++k) {
        int64_t n = std::min<int64_t>(chunk, T - s0);
        P.j0 = (uint32_t)s0;   // launch sample offset: keys the RNG streams through global_sample()
        P.n_items = (uint64_t)(n * n_slots);
        int64_t blocks_needed = ((int64_t)P.n_items + 255) / 256;
        int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)occ * s->cus, blocks_needed));
        // the camera kernel also zeroes the work counter (and, for the first chunk, the watchdog
        // flag) ahead of the trace launch: two fewer stream operations per frame
        P.cam_clears = 1 | (s0 == 0 ? 2 : 0);
        HIP_TRY(prt::launch_camera(P, (float4*)cx->rays.p, cam_fast ? nullptr : (float4*)cx->rays_o.p, stream));
        P.cam_clears = 0;
        if (timed) HIP_TRY(hipEventRecord(s->ev[2 * k], stream));
        DevBuf wclk;
        if (!s->wave_clock_path.empty()) {
            HIP_TRY(wclk.ensure(sizeof(unsigned long long) * 3 * (size_t)grid * (256 / 64)));
            HIP_TRY(hipMemsetAsync(wclk.p, 0, sizeof(unsigned long long) * 3 * (size_t)grid * 4, stream));
            P.wave_clock = (unsigned long long*)wclk.p;
        }
        HIP_TRY(prt::launch_trace(P, stack, var, grid, stats, stream));
        if (timed) HIP_TRY(hipEventRecord(s->ev[2 * k + 1], stream));
        if (P.wave_clock) {
            // diagnostic only: synchronous read-back, appended as (start, end, items) u64 triples
            std::vector<unsigned long long> h((size_t)grid * 4 * 3);
            HIP_TRY(hipMemcpyAsync(h.data(), wclk.p, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost,
                                   stream));
            HIP_TRY(hipStreamSynchronize(stream));
            if (FILE* f = std::fopen(s->wave_clock_path.c_str(), "ab")) {
                std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
                std::fclose(f);
            }
            P.wave_clock = nullptr;
        }
        // every frame overlapping the chunk, one launch: frame f sums its samples of [s0, s0 + n) in order
        {
            const int64_t f0 = s0 / spp, f1 = std::min<int64_t>(n_frames, (s0 + n + spp - 1) / spp);
            for (int64_t fa = f0; fa < f1; fa += 65535)
                HIP_TRY(prt::launch_reduce((const float*)cx->buf.p, d_acc, (int)n_slots, s0, n, spp, fa,
                                           std::min<int64_t>(65535, f1 - fa), out_pitch, accumulate, stream));
        }
    }
    return PRT_OK;
}

// ---------------------------------------------------------------- RCCL ----
// prt_render_multi's gather runs over RCCL.  librccl is resolved at first use with dlopen
// (by SONAME first, so a process that already loaded torch's RCCL shares that instance
// and its HIP runtime), which keeps libprt loadable on machines without RCCL: only
// prt_render_multi then fails, with PRT_ERR_RCCL.
struct Rccl {
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string why;
};

std::mutex g_comm_mu;   // guards g_rccl and g_comms
Rccl g_rccl;
bool g_rccl_tried = false;
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;   // per device list (root first)

const Rccl& rccl() {
    if (g_rccl_tried) return g_rccl;
    g_rccl_tried = true;
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
        if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
        g_rccl.why = std::string("librccl.so.1 not loadable: ") + (dlerror() ? dlerror() : "?");
        return g_rccl;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    g_rccl.comm_init_all = (decltype(g_rccl.comm_init_all))sym("ncclCommInitAll");
    g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))sym("ncclCommDestroy");
    g_rccl.group_start = (decltype(g_rccl.group_start))sym("ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))sym("ncclGroupEnd");
    g_rccl.send = (decltype(g_rccl.send))sym("ncclSend");
    g_rccl.recv = (decltype(g_rccl.recv))sym("ncclRecv");
    g_rccl.error_string = (decltype(g_rccl.error_string))sym("ncclGetErrorString");
    g_rccl.ok = g_rccl.comm_init_all && g_rccl.comm_destroy && g_rccl.group_start && g_rccl.group_end &&
                g_rccl.send && g_rccl.recv && g_rccl.error_string;
    if (!g_rccl.ok) g_rccl.why = "librccl lacks ncclCommInitAll / ncclSend / ncclRecv / group calls";
    return g_rccl;
}

#define RCCL_TRY(expr)                                                                           \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) return fail(PRT_ERR_RCCL, std::string(#expr) + ": " + R.error_string(r_)); \
    } while (0)

// 'latin' tile owner of device_scene.tile_owner: rank = (tx + s * ty) mod n with s the
// integer nearest 0.38 n that is coprime with n (every rank owns tiles in every row)
int latin_stride(int n) {
    int s = std::max(1, (int)std::lround(0.38 * n));
    auto gcd = [](int a, int b) { while (b) { int t = a % b; a = b; b = t; } return a; };
    while (gcd(s, n) != 1) ++s;
    return s;
}

// tile ids of a window, ascending (tiles of tw x th in the W-wide frame)
std::vector<int32_t> window_tiles(int W, int x0, int y0, int w, int h, int tw, int th) {
    const int tiles_x = (W + tw - 1) / tw;
    std::vector<int32_t> ids;
    for (int ty = y0 / th; ty <= (y0 + h - 1) / th; ++ty)
        for (int tx = x0 / tw; tx <= (x0 + w - 1) / tw; ++tx) ids.push_back(ty * tiles_x + tx);
    return ids;
}

}  // namespace

extern "C" {

int prt_abi_version(void) { return PRT_ABI_VERSION; }

const char* prt_last_error(void) { return g_err.c_str(); }

int prt_device_count(int* n) {
    if (!n) return fail(PRT_ERR_ARG, "n is NULL");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return PRT_OK;
}

int prt_bvh_build(const float* tri_v, int64_t n_tri, int32_t max_leaf, void** out_bvh) {
    if (!out_bvh || (n_tri > 0 && !tri_v)) return fail(PRT_ERR_ARG, "NULL argument");
    auto* b = new (std::nothrow) prt::BvhHost();
    if (!b) return fail(PRT_ERR_OOM, "host allocation failed");
    std::string err;
    try {
        if (!prt::build_bvh(tri_v, n_tri, max_leaf, b, &err)) { delete b; return fail(PRT_ERR_ARG, err); }
    } catch (const std::bad_alloc&) {
        delete b;
        return fail(PRT_ERR_OOM, "host allocation failed during BVH build");
    }
    *out_bvh = b;
    return PRT_OK;
}

int prt_bvh_info(void* bvh, int64_t* info6) {
    auto* b = (prt::BvhHost*)bvh;
    if (!b || !info6) return fail(PRT_ERR_ARG, "NULL argument");
    int32_t padbits;
    std::memcpy(&padbits, &b->pad, 4);
    info6[0] = b->n_nodes; info6[1] = b->depth; info6[2] = b->n_leaves; info6[3] = (int64_t)b->order.size();
    info6[4] = padbits; info6[5] = (int64_t)(b->sah_cost * 1000.0 + 0.5);
    return PRT_OK;
}

int prt_bvh_export(void* bvh, float* nodes, float* tris, int32_t* order) {
    auto* b = (prt::BvhHost*)bvh;
    if (!b) return fail(PRT_ERR_ARG, "NULL argument");
    if (nodes) std::memcpy(nodes, b->nodes.data(), sizeof(float) * b->nodes.size());
    if (tris) std::memcpy(tris, b->tris.data(), sizeof(float) * b->tris.size());
    if (order) std::memcpy(order, b->order.data(), sizeof(int32_t) * b->order.size());
    return PRT_OK;
}

void prt_bvh_destroy(void* bvh) { delete (prt::BvhHost*)bvh; }

int prt_scene_create(int device, const float* tri_v, const float* tri_n, const int32_t* tri_mat, int64_t n_tri,
                     const float* sph, const int32_t* sph_mat, int64_t n_sph, const float* mat, int32_t n_mat,
                     const int32_t* light_tri, const int32_t* light_off, int32_t n_light, const float* direct_rgb,
                     void** out_scene) {
    if (!out_scene) return fail(PRT_ERR_ARG, "out_scene is NULL");
    *out_scene = nullptr;
    if (n_tri < 0 || (n_tri > 0 && (!tri_v || !tri_n || !tri_mat))) return fail(PRT_ERR_ARG, "bad triangle arrays");
    if (n_sph < 0 || (n_sph > 0 && (!sph || !sph_mat))) return fail(PRT_ERR_ARG, "bad sphere arrays");
    for (int64_t k = 0; k < n_sph; ++k) {
        if (sph_mat[k] < 0 || sph_mat[k] >= n_mat) return fail(PRT_ERR_ARG, "sphere material id out of range");
        if (!(sph[4 * k + 3] > 0.0f)) return fail(PRT_ERR_ARG, "sphere radius must be > 0");
    }
    if (n_tri + n_sph >= ((int64_t)1 << 31)) return fail(PRT_ERR_ARG, "too many primitives");
    if (n_mat < 1 || !mat) return fail(PRT_ERR_ARG, "need at least one material");
    if (n_light < 1 || !light_off || !light_tri) return fail(PRT_ERR_ARG, "There is no lights!!! (n_light < 1)");
    for (int64_t i = 0; i < n_tri; ++i)
        if (tri_mat[i] < 0 || tri_mat[i] >= n_mat) return fail(PRT_ERR_ARG, "material id out of range at triangle " + std::to_string(i));
    if (light_off[0] != 0) return fail(PRT_ERR_ARG, "light_off[0] must be 0");
    for (int l = 0; l < n_light; ++l)
        if (light_off[l + 1] <= light_off[l]) return fail(PRT_ERR_ARG, "every light needs >= 1 triangle");
    for (int32_t k = 0; k < light_off[n_light]; ++k)
        if (light_tri[k] < 0 || light_tri[k] >= n_tri) return fail(PRT_ERR_ARG, "light triangle out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PRT_ERR_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(PRT_ERR_ARG, "device index out of range");

    prt::BvhHost bvh;
    std::string err;
    try {
        int max_leaf = 4;
        if (const char* ml = std::getenv("PRT_MAX_LEAF")) max_leaf = std::atoi(ml);
        if (!prt::build_bvh(tri_v, n_tri, max_leaf, &bvh, &err)) return fail(PRT_ERR_ARG, err);
    } catch (const std::bad_alloc&) {
        return fail(PRT_ERR_OOM, "host allocation failed during BVH build");
    }
    auto* s = new (std::nothrow) Scene();
    if (!s) return fail(PRT_ERR_OOM, "host allocation failed");
    s->device = device;
    s->n_tri = n_tri;
    s->n_nodes = bvh.n_nodes;
    s->depth = bvh.depth;
    s->n_light = n_light;
    s->n_mat = n_mat;
    if (direct_rgb) std::memcpy(s->direct_rgb, direct_rgb, sizeof(float) * 3);
    DeviceGuard g(device);
    int rc = PRT_OK;
    do {
        hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
        if (e != hipSuccess) { rc = fail(PRT_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e)); break; }
        std::vector<float> nm((size_t)std::max<int64_t>(n_tri, 1) * 4, 0.0f);
        for (int64_t i = 0; i < n_tri; ++i) {
            nm[4 * i] = tri_n[3 * i]; nm[4 * i + 1] = tri_n[3 * i + 1]; nm[4 * i + 2] = tri_n[3 * i + 2];
            nm[4 * i + 3] = bits_f(tri_mat[i]);
        }
        std::vector<float> fr((size_t)std::max<int64_t>(n_tri, 1) * 24, 0.0f);
        for (int64_t i = 0; i < n_tri; ++i) {
            F3 nn{tri_n[3 * i], tri_n[3 * i + 1], tri_n[3 * i + 2]};
            frame_rows(nn, fr.data() + 24 * i);
            frame_rows(F3{-nn.x, -nn.y, -nn.z}, fr.data() + 24 * i + 12);
        }
        int n_lt = light_off[n_light];
        s->n_lt = n_lt;
        std::vector<float> lv((size_t)n_lt * 16, 0.0f);
        for (int k = 0; k < n_lt; ++k) {
            int64_t t = light_tri[k];
            for (int c = 0; c < 3; ++c) {
                lv[16 * k + c] = tri_v[9 * t + c];
                lv[16 * k + 4 + c] = tri_v[9 * t + 3 + c];
                lv[16 * k + 8 + c] = tri_v[9 * t + 6 + c];
                lv[16 * k + 12 + c] = tri_n[3 * t + c];
            }
            lv[16 * k + 15] = bits_f(tri_mat[t]);
        }
        {
            prt::Bvh4Host b4;
            prt::collapse_bvh4(bvh, &b4);
            s->depth4 = b4.depth;
            s->n_node4_f4 = (int64_t)b4.nodes.size() / 4;
            s->stack4 = b4.stack_need <= 32 ? prt::stack_variant(b4.stack_need - 1) : 0;
            s->need4 = b4.stack_need;
            if ((rc = upload(s->nodes4, b4.nodes.data(), sizeof(float) * b4.nodes.size(), &s->device_bytes))) break;
            std::vector<float> q4;
            prt::quantize_bvh4(b4, bvh.pad, &q4);
            s->n_node4q_f4 = (int64_t)q4.size() / 4;
            if ((rc = upload(s->nodes4q, q4.data(), sizeof(float) * q4.size(), &s->device_bytes))) break;
        }
        if ((rc = upload(s->tris, bvh.tris.data(), sizeof(float) * bvh.tris.size(), &s->device_bytes))) break;
        if ((rc = upload(s->tri_nm, nm.data(), sizeof(float) * nm.size(), &s->device_bytes))) break;
        if ((rc = upload(s->tri_frame, fr.data(), sizeof(float) * fr.size(), &s->device_bytes))) break;
        if ((rc = upload(s->mats, mat, sizeof(float) * 8 * (size_t)n_mat, &s->device_bytes))) break;
        if ((rc = upload(s->light_v, lv.data(), sizeof(float) * lv.size(), &s->device_bytes))) break;
        if ((rc = upload(s->light_off, light_off, sizeof(int32_t) * (size_t)(n_light + 1), &s->device_bytes))) break;
        s->n_sph = n_sph;
        s->plain = n_sph == 0;
        for (int32_t i = 0; i < n_mat; ++i)
            if (mat[8 * i + 5] == 2.0f || mat[8 * i + 5] == 3.0f) s->plain = false;   // metal / dielectric
        // the shading quotients' cheap guards (prt_device.h lambert_div / nee_div) assume albedos and
        // emitters in [2^-40, 2^40] and face normals of length in [0.5, 2]; other scenes keep div3's guard
        s->shade_fast = true;
        for (int32_t i = 0; i < n_mat && s->shade_fast; ++i)
            for (int c = 0; c < 3; ++c) {
                const float r = mat[8 * i + c];
                if (!(r >= 0x1p-40f && r <= 0x1p40f)) s->shade_fast = false;
            }
        for (int64_t i = 0; i < n_tri && s->shade_fast; ++i) {
            const double x = tri_n[3 * i], y = tri_n[3 * i + 1], z = tri_n[3 * i + 2];
            const double l2 = x * x + y * y + z * z;
            if (!(l2 >= 0.25 && l2 <= 4.0)) s->shade_fast = false;
        }
        if ((rc = upload(s->sph, sph, sizeof(float) * 4 * (size_t)n_sph, &s->device_bytes))) break;
        if ((rc = upload(s->sph_mat, sph_mat, sizeof(int32_t) * (size_t)n_sph, &s->device_bytes))) break;
        if ((e = s->work.ensure(64)) != hipSuccess || (e = s->stats.ensure(8 * kStatWords)) != hipSuccess) {
            rc = fail(PRT_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
            break;
        }
        // the hit-query watchdog flag is read by prt_check_faults before any hit query ran
        if ((e = hipMemset(s->work.p, 0, 64)) != hipSuccess) { rc = fail(PRT_ERR_HIP, hipGetErrorString(e)); break; }
        hipDeviceProp_t prop;
        if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) { rc = fail(PRT_ERR_HIP, hipGetErrorString(e)); break; }
        s->cus = prop.multiProcessorCount;
        s->n_tri_f4 = (int64_t)bvh.tris.size() / 4;
        if (const char* le = std::getenv("PRT_LEAF_EXIT")) s->leaf_exit = std::max(0, std::min(64, std::atoi(le)));
        if (const char* lb = std::getenv("PRT_LEAF_BREAK")) s->leaf_break = std::max(0, std::min(64, std::atoi(lb)));
        if (const char* wc = std::getenv("PRT_WAVE_CLOCK")) s->wave_clock_path = wc;
        if (const char* gt = std::getenv("PRT_GUARD_TRIPS"))
            s->guard_trips = (uint32_t)std::max(1LL, std::min((long long)UINT32_MAX, std::atoll(gt)));
        if (const char* rm = std::getenv("PRT_RESUME_MIN")) s->resume_min = std::max(1, std::min(64, std::atoi(rm)));
        if (const char* sl = std::getenv("PRT_SPILL_LDS")) {
            int v = std::atoi(sl);
            s->spill_lds = v == 4 ? 4 : v == 32 ? 32 : 16;
        }
        {
            prt::TraceParams Q;
            std::memset(&Q, 0, sizeof(Q));
            int var = default_variant(s);
            scene_sizes(s, Q);
            Q.lds_stack = s->need4;
            int stk = variant_stack(s, var);
            s->blocks_per_cu = std::max(1, prt::trace_blocks_per_cu(stk, var, false, prt::trace_smem_bytes(stk, var, Q)));
        }
        if (const char* cb = std::getenv("PRT_CHUNK_BYTES")) {
            s->chunk_bytes = (size_t)std::max(1LL << 20, std::atoll(cb));
        } else {
            // the default budget takes at most a quarter of the memory free at scene creation (16 GiB
            // of an idle MI355X's 288 GB); enqueue_render also caps it by the memory free when a
            // render stream's buffers grow
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
                s->chunk_bytes = std::max<size_t>((size_t)1 << 28, std::min(s->chunk_bytes, free_b / 4));
        }
    } while (0);
    if (rc != PRT_OK) { destroy_scene(s); return rc; }
    *out_scene = s;
    return PRT_OK;
}

int prt_scene_info(void* scene, int64_t* info8) {
    auto* s = (Scene*)scene;
    if (!s || !info8) return fail(PRT_ERR_ARG, "NULL argument");
    info8[0] = s->device; info8[1] = s->n_tri; info8[2] = s->n_nodes; info8[3] = s->depth;
    info8[4] = s->stack4; info8[5] = (int64_t)s->device_bytes; info8[6] = s->blocks_per_cu; info8[7] = s->cus;
    return PRT_OK;
}

int prt_closest_hits(void* scene, const float* rays, int64_t n, uint32_t flags, int32_t* hit_id, float* hit_t) {
    auto* s = (Scene*)scene;
    if (!s || (n > 0 && (!rays || !hit_id || !hit_t))) return fail(PRT_ERR_ARG, "NULL argument");
    if (n < 0) return fail(PRT_ERR_ARG, "n < 0");
    if (n == 0) return PRT_OK;
    if (s->need4 > 64) return fail(PRT_ERR_ARG, "BVH4 too deep for the hit-query kernel");
    DeviceGuard g(s->device);
    const bool quant = (flags & PRT_HITS_QUANTIZED) != 0, any = (flags & PRT_HITS_ANY) != 0;
    prt::TraceParams P;
    std::memset(&P, 0, sizeof(P));
    P.nodes = (const float4*)(quant ? s->nodes4q.p : s->nodes4.p);
    P.tris = (const float4*)s->tris.p;
    P.n_tri = (int)s->n_tri;
    P.n_sph = (int)s->n_sph;
    P.sph = (const float4*)s->sph.p;
    DevBuf d_rays, d_id, d_t;
    HIP_TRY(d_rays.ensure(sizeof(float) * 8 * (size_t)n));
    HIP_TRY(d_id.ensure(sizeof(int32_t) * (size_t)n));
    HIP_TRY(d_t.ensure(sizeof(float) * (size_t)n));
    P.fault = (int*)((char*)s->work.p + kFaultOffset);
    P.guard_trips = s->guard_trips;
    HIP_TRY(hipMemsetAsync(P.fault, 0, sizeof(int), s->stream));
    HIP_TRY(hipMemcpyAsync(d_rays.p, rays, sizeof(float) * 8 * (size_t)n, hipMemcpyHostToDevice, s->stream));
    HIP_TRY(prt::launch_hits(P, quant, any, 64, (const float4*)d_rays.p, n, (int*)d_id.p, (float*)d_t.p, s->stream));
    HIP_TRY(hipMemcpyAsync(hit_id, d_id.p, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipMemcpyAsync(hit_t, d_t.p, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (take_fault(s) != 0) return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    return PRT_OK;
}

int prt_hit_all(void* scene, const float* rays, int64_t n, uint64_t seed, uint32_t flags, float* out16) {
    auto* s = (Scene*)scene;
    if (!s || (n > 0 && (!rays || !out16))) return fail(PRT_ERR_ARG, "NULL argument");
    if (n < 0) return fail(PRT_ERR_ARG, "n < 0");
    if (flags & ~PRT_HITS_QUANTIZED) return fail(PRT_ERR_ARG, "prt_hit_all takes only PRT_HITS_QUANTIZED");
    if (n == 0) return PRT_OK;
    if (s->need4 > 64) return fail(PRT_ERR_ARG, "BVH4 too deep for the hit-query kernel");
    DeviceGuard g(s->device);
    const bool quant = (flags & PRT_HITS_QUANTIZED) != 0;
    prt::TraceParams P;
    scene_params(s, P);
    if (quant) P.nodes = (const float4*)s->nodes4q.p;
    P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
    P.fault = (int*)((char*)s->work.p + kFaultOffset);
    DevBuf d_rays, d_id, d_t, d_out;
    HIP_TRY(d_rays.ensure(sizeof(float) * 8 * (size_t)n));
    HIP_TRY(d_id.ensure(sizeof(int32_t) * (size_t)n));
    HIP_TRY(d_t.ensure(sizeof(float) * (size_t)n));
    HIP_TRY(d_out.ensure(sizeof(float) * 16 * (size_t)n));
    HIP_TRY(hipMemsetAsync(P.fault, 0, sizeof(int), s->stream));
    HIP_TRY(hipMemcpyAsync(d_rays.p, rays, sizeof(float) * 8 * (size_t)n, hipMemcpyHostToDevice, s->stream));
    HIP_TRY(prt::launch_hits(P, quant, false, 64, (const float4*)d_rays.p, n, (int*)d_id.p, (float*)d_t.p, s->stream));
    HIP_TRY(prt::launch_hit_shade(P, (const float4*)d_rays.p, n, (const int*)d_id.p, (const float*)d_t.p,
                                  (float*)d_out.p, s->stream));
    HIP_TRY(hipMemcpyAsync(out16, d_out.p, sizeof(float) * 16 * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (take_fault(s) != 0) return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    return PRT_OK;
}

int prt_trace_rays(void* scene, const float* rays, int64_t n, int depth, uint64_t seed, uint32_t flags,
                   float* out_rgb) {
    auto* s = (Scene*)scene;
    if (!s || (n > 0 && (!rays || !out_rgb))) return fail(PRT_ERR_ARG, "NULL argument");
    if (n < 0 || depth < 0) return fail(PRT_ERR_ARG, "n and depth must be >= 0");
    if (flags & (PRT_FLAG_NO_PRIMARY_KERNEL | PRT_FLAG_TIME))
        return fail(PRT_ERR_ARG, "prt_trace_rays: PRT_FLAG_NO_PRIMARY_KERNEL / PRT_FLAG_TIME do not apply");
    if (n == 0) return PRT_OK;
    if (n >= ((int64_t)1 << 31)) return fail(PRT_ERR_ARG, "too many rays in one call (< 2^31)");
    DeviceGuard g(s->device);
    if (depth == 0) {
        std::memset(out_rgb, 0, sizeof(float) * 3 * (size_t)n);
        return PRT_OK;
    }
    RenderCtx* cx = ctx_for(s, s->stream);
    if (!cx) return fail(PRT_ERR_OOM, "render context allocation failed");
    // the rays as one "sample" of a frame of 64 x 1 tiles: item = slot = ray index (every chunk
    // of 64 items one tile); the trace kernel's tile origins are (0, tile)
    constexpr int64_t kRowRays = 64;
    const int64_t n_pad = (n + kRowRays - 1) / kRowRays * kRowRays;
    const int64_t n_tiles = n_pad / kRowRays;
    if (n_tiles > 65535) return fail(PRT_ERR_ARG, "too many rays in one call (<= 65535 x 64)");
    std::vector<uint32_t> origins((size_t)n_tiles);
    for (int64_t t = 0; t < n_tiles; ++t) origins[(size_t)t] = (uint32_t)t;
    if (origins != cx->tile_host) {
        // enqueued on the context's stream, behind any render still running there (an unsynchronised
        // prt_render_tiles_device reads the old origins until it ends); the host copy lives in
        // cx->tile_host until the next upload, as enqueue_render's
        HIP_TRY(cx->tiles.ensure(sizeof(uint32_t) * (size_t)n_tiles));
        HIP_TRY(hipMemcpyAsync(cx->tiles.p, origins.data(), sizeof(uint32_t) * (size_t)n_tiles,
                               hipMemcpyHostToDevice, cx->stream));
        cx->tile_host.swap(origins);
    }
    DevBuf d_in, d_org, d_out;
    HIP_TRY(d_in.ensure(sizeof(float) * 8 * (size_t)n));
    HIP_TRY(d_org.ensure(sizeof(float) * 4 * (size_t)n_pad));
    HIP_TRY(d_out.ensure(sizeof(float) * 3 * (size_t)n_pad));
    HIP_TRY(cx->rays.ensure(sizeof(float) * 4 * (size_t)n_pad));
    HIP_TRY(hipMemcpyAsync(d_in.p, rays, sizeof(float) * 8 * (size_t)n, hipMemcpyHostToDevice, s->stream));
    prt::TraceParams P;
    scene_params(s, P);
    P.rays = (const float4*)cx->rays.p;
    P.ray_o = (const float4*)d_org.p;
    P.W = (int)kRowRays; P.H = (int)n_tiles;
    P.wm1 = (float)(kRowRays - 1); P.hm1 = (float)std::max<int64_t>(n_tiles - 1, 1);
    P.log_tw = 6;
    P.log_tpx = 6;
    P.tile_xy = (const uint32_t*)cx->tiles.p;
    P.n_slots = (int)n_pad;
    P.s0 = 0;
    P.n_items = (uint64_t)n_pad;
    P.depth = depth;
    P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
    P.work = (uint32_t*)cx->work.p;
    P.fault = (int*)((char*)cx->work.p + kFaultOffset);
    P.out = (float*)d_out.p;
    int var = 0, stack = 0, occ = 0;
    if (int rc = trace_setup(s, cx, flags, n_pad, P, &var, &stack, &occ)) return rc;
    const bool stats = (flags & PRT_FLAG_STATS) != 0;
    if (stats) HIP_TRY(hipMemsetAsync(s->stats.p, 0, kStatWords * sizeof(unsigned long long), s->stream));
    HIP_TRY(hipMemsetAsync(cx->work.p, 0, 64, s->stream));   // work counter and watchdog flag
    HIP_TRY(prt::launch_rays_prep(P, (const float*)d_in.p, n, n_pad, (float4*)cx->rays.p, (float4*)d_org.p, s->stream));
    const int64_t blocks_needed = (n_pad + 255) / 256;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)occ * s->cus, blocks_needed));
    HIP_TRY(prt::launch_trace(P, stack, var, grid, stats, s->stream));
    HIP_TRY(hipMemcpyAsync(out_rgb, d_out.p, sizeof(float) * 3 * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (take_fault_at(cx->work) != 0)
        return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    return PRT_OK;
}

int prt_camera_rays(void* scene, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids,
                    int n_tiles, int first_sample, int spp, uint64_t seed, float* out8) {
    auto* s = (Scene*)scene;
    if (int rc = check_render_args(s, cam, W, H, tw, th, tile_ids, n_tiles, spp, 1)) return rc;
    if (first_sample < 0 || (int64_t)first_sample + spp > INT32_MAX)
        return fail(PRT_ERR_ARG, "sample indices must stay in [0, 2^31)");
    const int64_t n_slots = (int64_t)n_tiles * tw * th, n = n_slots * spp;
    if (n == 0) return PRT_OK;
    if (!out8) return fail(PRT_ERR_ARG, "out8 is NULL");
    if (n >= ((int64_t)1 << 31)) return fail(PRT_ERR_ARG, "too many rays in one call (< 2^31)");
    DeviceGuard g(s->device);
    const int tiles_x = (W + tw - 1) / tw;
    std::vector<uint32_t> origins((size_t)n_tiles);
    for (int i = 0; i < n_tiles; ++i)
        origins[(size_t)i] = ((uint32_t)((tile_ids[i] % tiles_x) * tw) << 16) | (uint32_t)((tile_ids[i] / tiles_x) * th);
    DevBuf d_tiles, d_rays, d_org;
    HIP_TRY(d_tiles.ensure(sizeof(uint32_t) * (size_t)n_tiles));
    HIP_TRY(d_rays.ensure(16 * (size_t)n));
    HIP_TRY(d_org.ensure(16 * (size_t)n));
    HIP_TRY(hipMemcpyAsync(d_tiles.p, origins.data(), sizeof(uint32_t) * (size_t)n_tiles, hipMemcpyHostToDevice,
                           s->stream));
    prt::TraceParams P;
    scene_params(s, P);
    camera_params(P, cam, W, H, tw, th);
    P.tile_xy = (const uint32_t*)d_tiles.p;
    P.n_slots = (int)n_slots;
    P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
    P.s0 = first_sample;
    P.j0 = 0;
    // one frame of spp samples starting at first_sample, as enqueue_render keys it (global_sample
    // divides by frame_spp)
    P.frame_spp = (uint32_t)spp;
    P.frame_stride = 0;
    P.n_items = (uint64_t)n;
    P.cam_clears = 0;
    // slots outside the frame (partial edge tiles) get no ray from the camera kernel: their rows are
    // returned as zeros, not as uninitialised device memory
    HIP_TRY(hipMemsetAsync(d_rays.p, 0, 16 * (size_t)n, s->stream));
    if (!P.cam_fast) HIP_TRY(hipMemsetAsync(d_org.p, 0, 16 * (size_t)n, s->stream));
    HIP_TRY(prt::launch_camera(P, (float4*)d_rays.p, P.cam_fast ? nullptr : (float4*)d_org.p, s->stream));
    std::vector<float> r((size_t)n * 4), o(P.cam_fast ? 0 : (size_t)n * 4);
    HIP_TRY(hipMemcpyAsync(r.data(), d_rays.p, 16 * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    if (!P.cam_fast) HIP_TRY(hipMemcpyAsync(o.data(), d_org.p, 16 * (size_t)n, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const int64_t tpx = (int64_t)tw * th;
    for (int64_t i = 0; i < n; ++i) {
        float* q = out8 + 8 * i;
        // slot -> pixel as the kernels map it (pixel_of): tile-major, then row-major within the tile
        const int64_t slot = i % n_slots, loc = slot % tpx;
        const uint32_t xy0 = origins[(size_t)(slot / tpx)];
        const bool in_frame = (int64_t)(xy0 >> 16) + loc % tw < W && (int64_t)(xy0 & 0xFFFFu) + loc / tw < H;
        for (int k = 0; k < 3; ++k) {
            q[k] = !in_frame ? 0.0f : P.cam_fast ? P.cam_o[k] : o[(size_t)(4 * i + k)];
            q[4 + k] = r[(size_t)(4 * i + k)];
        }
        q[3] = r[(size_t)(4 * i + 3)];   // the RNG state after the camera's draws (u32 bits)
        q[7] = 0.0f;
    }
    return PRT_OK;
}

int prt_scene_kernel(void* scene, int32_t* out4) { return prt_launch_kernel(scene, INT64_MAX, 0, out4); }

int prt_launch_kernel(void* scene, int64_t n_items, uint32_t flags, int32_t* out4) {
    auto* s = (Scene*)scene;
    if (!s || !out4) return fail(PRT_ERR_ARG, "NULL argument");
    if (n_items < 0) return fail(PRT_ERR_ARG, "n_items < 0");
    int var = launch_variant(s, flags, n_items);
    out4[0] = var;
    out4[1] = 4;
    out4[2] = (prt::variant_uses_lds(var) ? 1 : 0) | (prt::variant_quantized(var) ? 2 : 0);
    // the pooled kernel's LDS stack is sized to the BVH4's exact bound (P.lds_stack = need4)
    out4[3] = prt::variant_pool(var) ? s->need4 : variant_stack(s, var);
    return PRT_OK;
}

void prt_scene_destroy(void* scene) { destroy_scene((Scene*)scene); }

int prt_render_tiles(void* scene, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids, int n_tiles,
                     int spp, int depth, uint64_t seed, uint32_t flags, float* out_sum, uint64_t* stats) {
    auto* s = (Scene*)scene;
    int rc = check_render_args(s, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth);
    if (rc) return rc;
    if (!out_sum) return fail(PRT_ERR_ARG, "out_sum is NULL");
    DeviceGuard g(s->device);
    const int64_t n_slots = (int64_t)n_tiles * tw * th;
    RenderCtx* cx = ctx_for(s, s->stream);
    if (!cx) return fail(PRT_ERR_OOM, "render context allocation failed");
    HIP_TRY(cx->acc.ensure(std::max<size_t>(16, sizeof(float) * 3 * (size_t)n_slots)));
    if ((rc = enqueue_render(s, cx, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth, seed, flags, (float*)cx->acc.p)))
        return rc;
    if (n_slots)
        HIP_TRY(hipMemcpyAsync(out_sum, cx->acc.p, sizeof(float) * 3 * (size_t)n_slots, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (take_fault_at(cx->work) != 0)
        return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    if (stats) {
        if (flags & PRT_FLAG_STATS) {
            unsigned long long h[4];
            HIP_TRY(hipMemcpy(h, s->stats.p, sizeof(h), hipMemcpyDeviceToHost));
            for (int i = 0; i < 4; ++i) stats[i] = h[i];
        } else {
            std::memset(stats, 0, 4 * sizeof(uint64_t));
        }
    }
    return PRT_OK;
}

int prt_render_tiles_accumulate(void* scene, const float* cam, int W, int H, int tw, int th,
                                const int32_t* tile_ids, int n_tiles, int first_sample, int spp, int depth,
                                uint64_t seed, uint32_t flags, float* io_sum) {
    auto* s = (Scene*)scene;
    int rc = check_render_args(s, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth);
    if (rc) return rc;
    if (!io_sum && n_tiles > 0) return fail(PRT_ERR_ARG, "io_sum is NULL");
    if (first_sample < 0 || (int64_t)first_sample + spp > INT32_MAX)
        return fail(PRT_ERR_ARG, "first_sample must be >= 0 and first_sample + spp < 2^31");
    DeviceGuard g(s->device);
    const int64_t n_slots = (int64_t)n_tiles * tw * th;
    if (n_slots == 0) return PRT_OK;
    RenderCtx* cx = ctx_for(s, s->stream);
    if (!cx) return fail(PRT_ERR_OOM, "render context allocation failed");
    const size_t bytes = sizeof(float) * 3 * (size_t)n_slots;
    HIP_TRY(cx->acc.ensure(std::max<size_t>(16, bytes)));
    HIP_TRY(hipMemcpyAsync(cx->acc.p, io_sum, bytes, hipMemcpyHostToDevice, s->stream));
    if ((rc = enqueue_render(s, cx, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth, seed, flags, (float*)cx->acc.p,
                             first_sample, true)))
        return rc;
    HIP_TRY(hipMemcpyAsync(io_sum, cx->acc.p, bytes, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (take_fault_at(cx->work) != 0)
        return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    return PRT_OK;
}

int prt_render_tiles_device(void* scene, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids,
                            int n_tiles, int spp, int depth, uint64_t seed, uint32_t flags, float* d_out_sum,
                            void* stream) {
    auto* s = (Scene*)scene;
    int rc = check_render_args(s, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth);
    if (rc) return rc;
    if (!d_out_sum && n_tiles > 0) return fail(PRT_ERR_ARG, "d_out_sum is NULL");
    DeviceGuard g(s->device);
    RenderCtx* cx = ctx_for(s, stream ? (hipStream_t)stream : s->stream);
    if (!cx) return fail(PRT_ERR_OOM, "render context allocation failed");
    return enqueue_render(s, cx, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth, seed, flags, d_out_sum);
}

int prt_render_frames_device(void* scene, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids,
                             int n_tiles, int spp, int depth, uint64_t seed, int n_frames, int frame_stride,
                             uint32_t flags, float* d_out_sums, int64_t out_pitch, void* stream) {
    auto* s = (Scene*)scene;
    int rc = check_render_args(s, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth);
    if (rc) return rc;
    if (n_frames < 1) return fail(PRT_ERR_ARG, "n_frames must be >= 1");
    if (frame_stride < 0) return fail(PRT_ERR_ARG, "frame_stride must be >= 0");
    if ((int64_t)(n_frames - 1) * frame_stride + spp > INT32_MAX || (int64_t)n_frames * spp > INT32_MAX)
        return fail(PRT_ERR_ARG, "sample indices must stay below 2^31");
    if (!d_out_sums && n_tiles > 0) return fail(PRT_ERR_ARG, "d_out_sums is NULL");
    if (out_pitch != 0 && out_pitch < 3 * (int64_t)n_tiles * tw * th)
        return fail(PRT_ERR_ARG, "out_pitch must be 0 (packed frames) or >= n_tiles * tw * th * 3 floats");
    DeviceGuard g(s->device);
    RenderCtx* cx = ctx_for(s, stream ? (hipStream_t)stream : s->stream);
    if (!cx) return fail(PRT_ERR_OOM, "render context allocation failed");
    return enqueue_render(s, cx, cam, W, H, tw, th, tile_ids, n_tiles, spp, depth, seed, flags, d_out_sums, 0, false,
                          n_frames, frame_stride, out_pitch);
}

int prt_kernel_timing(void* scene, double* ms_total, int64_t* launches) {
    auto* s = (Scene*)scene;
    if (!s || !ms_total || !launches) return fail(PRT_ERR_ARG, "NULL argument");
    DeviceGuard g(s->device);
    double tot = 0.0;
    for (int k = 0; k + 1 < s->ev_used; k += 2) {
        HIP_TRY(hipEventSynchronize(s->ev[k + 1]));
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev[k], s->ev[k + 1]));
        tot += ms;
    }
    *ms_total = tot;
    *launches = s->ev_used / 2;
    if (take_render_faults(s) != 0) {
        s->ev_used = 0;
        return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    }
    s->ev_used = 0;
    return PRT_OK;
}

int prt_selftest_guards(int device, uint64_t* counts16) {
    if (!counts16) return fail(PRT_ERR_ARG, "NULL argument");
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return fail(PRT_ERR_HIP, "no such HIP device");
    DeviceGuard g(device);
    DevBuf d;
    HIP_TRY(d.ensure(16 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(d.p, 0, 16 * sizeof(unsigned long long)));
    HIP_TRY(prt::launch_guard_selftest((unsigned long long*)d.p, nullptr));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[16];
    HIP_TRY(hipMemcpy(h, d.p, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < 16; ++i) counts16[i] = h[i];
    return PRT_OK;
}

int prt_selftest_rcp(int device, uint64_t* mismatches8) {
    if (!mismatches8) return fail(PRT_ERR_ARG, "NULL argument");
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return fail(PRT_ERR_HIP, "no such HIP device");
    DeviceGuard g(device);
    DevBuf d;
    HIP_TRY(d.ensure(8 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(d.p, 0, 8 * sizeof(unsigned long long)));
    HIP_TRY(prt::launch_rcp_selftest((unsigned long long*)d.p, nullptr));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[8];
    HIP_TRY(hipMemcpy(h, d.p, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; ++i) mismatches8[i] = h[i];
    return PRT_OK;
}

int prt_check_faults(void* scene) {
    auto* s = (Scene*)scene;
    if (!s) return fail(PRT_ERR_ARG, "NULL argument");
    DeviceGuard g(s->device);
    // every stream a render was enqueued on: the device-wide synchronisation also covers
    // streams the caller owns (torch streams) without holding their handles past their life
    HIP_TRY(hipDeviceSynchronize());
    if ((take_render_faults(s) | take_fault(s)) != 0)
        return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    return PRT_OK;
}

int prt_last_stats(void* scene, uint64_t* stats4) {
    auto* s = (Scene*)scene;
    if (!s || !stats4) return fail(PRT_ERR_ARG, "NULL argument");
    DeviceGuard g(s->device);
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[4];
    HIP_TRY(hipMemcpy(h, s->stats.p, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) stats4[i] = h[i];
    return PRT_OK;
}

int prt_diag_words(void* scene, uint64_t* out, int n) {
    auto* s = (Scene*)scene;
    if (!s || !out || n < 0) return fail(PRT_ERR_ARG, "NULL argument or n < 0");
    DeviceGuard g(s->device);
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[kStatWords];
    HIP_TRY(hipMemcpy(h, s->stats.p, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) out[i] = i < kStatWords ? h[i] : 0;
    return PRT_OK;
}

int prt_diag_stats(void* scene, uint64_t* stats16) {
    auto* s = (Scene*)scene;
    if (!s || !stats16) return fail(PRT_ERR_ARG, "NULL argument");
    DeviceGuard g(s->device);
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[kStatWords];
    HIP_TRY(hipMemcpy(h, s->stats.p, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < 16; ++i) stats16[i] = h[i];
    return PRT_OK;
}

int prt_render(void* scene, const float* cam, int W, int H, int x0, int y0, int w, int h, int spp, int depth,
               uint64_t seed, uint32_t flags, float* out_sum, uint64_t* stats) {
    auto* s = (Scene*)scene;
    if (!s) return fail(PRT_ERR_ARG, "scene is NULL");
    if (w < 1 || h < 1 || x0 < 0 || y0 < 0 || (int64_t)x0 + w > W || (int64_t)y0 + h > H)
        return fail(PRT_ERR_ARG, "window [x0, x0+w) x [y0, y0+h) must be non-empty and inside the W x H frame");
    if (!out_sum) return fail(PRT_ERR_ARG, "out_sum is NULL");
    // 8 x 8 tiles: one wave's 64 work items cover one square tile (coherent rays), and a
    // window wastes at most a 7-pixel border of its edge tiles
    constexpr int kT = 8;
    std::vector<int32_t> ids = window_tiles(W, x0, y0, w, h, kT, kT);
    int rc = check_render_args(s, cam, W, H, kT, kT, ids.data(), (int)ids.size(), spp, depth);
    if (rc) return rc;
    DeviceGuard g(s->device);
    const int64_t n_slots = (int64_t)ids.size() * kT * kT;
    RenderCtx* cx = ctx_for(s, s->stream);
    if (!cx) return fail(PRT_ERR_OOM, "render context allocation failed");
    HIP_TRY(cx->acc.ensure(sizeof(float) * 3 * (size_t)n_slots));
    const size_t out_bytes = sizeof(float) * 3 * (size_t)w * (size_t)h;
    HIP_TRY(s->frame.ensure(out_bytes));
    if ((rc = enqueue_render(s, cx, cam, W, H, kT, kT, ids.data(), (int)ids.size(), spp, depth, seed, flags,
                             (float*)cx->acc.p)))
        return rc;
    HIP_TRY(prt::launch_scatter((const float*)cx->acc.p, (const uint32_t*)cx->tiles.p, (int)n_slots, 3, 6, x0, y0, w,
                                h, (float*)s->frame.p, s->stream));
    HIP_TRY(hipMemcpyAsync(out_sum, s->frame.p, out_bytes, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (take_fault_at(cx->work) != 0)
        return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped (corrupt acceleration structure?)");
    if (stats) {
        std::memset(stats, 0, 4 * sizeof(uint64_t));
        if (flags & PRT_FLAG_STATS) {
            unsigned long long hs[4];
            HIP_TRY(hipMemcpy(hs, s->stats.p, sizeof(hs), hipMemcpyDeviceToHost));
            for (int i = 0; i < 4; ++i) stats[i] = hs[i];
        }
    }
    return PRT_OK;
}

// shared by prt_scatter_tiles / prt_scatter_frames: argument checks and the (cached) upload of the
// tile origins; then one scatter launch over n_tiles * tw * th slots
static int scatter_enqueue(void* scene, const float* d_packed, const int32_t* tile_ids, int n_tiles, int tw, int th,
                           int W, int H, int group_tiles, int64_t group_pitch, int n_frames, int64_t src_fpitch,
                           float* d_frame, int64_t dst_fpitch, void* stream) {
    auto* s = (Scene*)scene;
    if (!s) return fail(PRT_ERR_ARG, "scene is NULL");
    if (n_tiles < 0 || (n_tiles > 0 && (!tile_ids || !d_packed || !d_frame))) return fail(PRT_ERR_ARG, "NULL argument");
    if (tw < 1 || th < 1 || (tw & (tw - 1)) || (th & (th - 1)) || (int64_t)tw * th > (1 << 20))
        return fail(PRT_ERR_ARG, "tile width/height must be powers of two with tw*th <= 2^20");
    if (W < 1 || H < 1 || W > 65535 || H > 65535) return fail(PRT_ERR_ARG, "frame must be 1..65535 pixels per side");
    const int tiles_x = (W + tw - 1) / tw, tiles_y = (H + th - 1) / th;
    for (int i = 0; i < n_tiles; ++i)
        if (tile_ids[i] < -1 || tile_ids[i] >= tiles_x * tiles_y)
            return fail(PRT_ERR_ARG, "tile id out of range: " + std::to_string(tile_ids[i]));
    if ((int64_t)n_tiles * tw * th >= ((int64_t)1 << 31)) return fail(PRT_ERR_ARG, "too many slots in one call");
    if (n_tiles == 0) return PRT_OK;
    DeviceGuard g(s->device);
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    // tile origins (x0 << 16 | y0); a padding slot (id -1) gets x0 = 0xFFFF, past any frame's
    // width (<= 65535), so the kernel drops its pixels
    std::vector<uint32_t> xy((size_t)n_tiles);
    for (int i = 0; i < n_tiles; ++i)
        xy[(size_t)i] = tile_ids[i] < 0 ? 0xFFFF0000u
                                        : ((uint32_t)((tile_ids[i] % tiles_x) * tw) << 16) |
                                              (uint32_t)((tile_ids[i] / tiles_x) * th);
    // uploaded only when they differ from the last call's (a bench or an animation scatters the
    // same tile set every frame): a steady-state frame then neither copies nor waits on the host
    if (xy != s->scatter_xy_host) {
        // earlier scatters (on any stream) may still read the device copy, and the previous
        // upload its host copy: a changed tile set waits for the device once
        if (s->scatter_ev) HIP_TRY(hipDeviceSynchronize());
        else HIP_TRY(hipEventCreateWithFlags(&s->scatter_ev, hipEventDisableTiming));
        HIP_TRY(s->scatter_xy.ensure(sizeof(uint32_t) * (size_t)n_tiles));
        s->scatter_xy_host.swap(xy);
        HIP_TRY(hipMemcpyAsync(s->scatter_xy.p, s->scatter_xy_host.data(), sizeof(uint32_t) * (size_t)n_tiles,
                               hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(s->scatter_ev, st));
    } else if (hipEventQuery(s->scatter_ev) != hipSuccess) {
        // same tile set, uploaded on a stream that may not have reached the copy yet
        HIP_TRY(hipStreamWaitEvent(st, s->scatter_ev, 0));
    }
    const int log_tw = __builtin_ctz((unsigned)tw), log_tpx = __builtin_ctz((unsigned)(tw * th));
    HIP_TRY(prt::launch_scatter_frames(d_packed, (const uint32_t*)s->scatter_xy.p, n_tiles * tw * th,
                                       group_tiles * tw * th, group_pitch, n_frames, src_fpitch, dst_fpitch, log_tw,
                                       log_tpx, 0, 0, W, H, d_frame, st));
    return PRT_OK;
}

int prt_scatter_tiles(void* scene, const float* d_packed, const int32_t* tile_ids, int n_tiles, int tw, int th,
                      int W, int H, float* d_frame, void* stream) {
    return scatter_enqueue(scene, d_packed, tile_ids, n_tiles, tw, th, W, H, std::max(n_tiles, 1), 0, 1, 0, d_frame, 0,
                           stream);
}

int prt_scatter_frames(void* scene, const float* d_packed, const int32_t* tile_ids, int n_groups, int group_tiles,
                       int64_t group_pitch, int tw, int th, int W, int H, int n_frames, int64_t src_frame_pitch,
                       float* d_frames, void* stream) {
    if (n_groups < 0 || group_tiles < 1 || n_frames < 1 || n_frames > 65535)
        return fail(PRT_ERR_ARG, "need n_groups >= 0, group_tiles >= 1 and 1 <= n_frames <= 65535");
    const int64_t slot_f = (int64_t)tw * th * 3;
    if (group_pitch < 0 || src_frame_pitch < 0 || (n_groups > 1 && group_pitch < group_tiles * slot_f) ||
        (n_frames > 1 && src_frame_pitch < group_tiles * slot_f))
        return fail(PRT_ERR_ARG, "group_pitch / src_frame_pitch must hold a group's tiles");
    // a group holds all n_frames frames of its tiles: frame f of group g must not reach into group g + 1
    // 
    if (n_groups > 1 && group_pitch < (int64_t)(n_frames - 1) * src_frame_pitch + group_tiles * slot_f)
        return fail(PRT_ERR_ARG, "group_pitch must hold n_frames frames of a group at src_frame_pitch");
    if ((int64_t)n_groups * group_tiles >= ((int64_t)1 << 31)) return fail(PRT_ERR_ARG, "too many tiles");
    return scatter_enqueue(scene, d_packed, tile_ids, n_groups * group_tiles, tw, th, W, H, group_tiles, group_pitch,
                           n_frames, src_frame_pitch, d_frames, 3 * (int64_t)W * H, stream);
}

int prt_render_multi(void* const* scenes, int n_scenes, const float* cam, int W, int H, int tile, int spp, int depth,
                     uint64_t seed, uint32_t flags, float* out_frame) {
    if (!scenes || n_scenes < 1) return fail(PRT_ERR_ARG, "need at least one scene handle");
    if (!out_frame) return fail(PRT_ERR_ARG, "out_frame is NULL");
    std::vector<Scene*> sc((size_t)n_scenes);
    std::vector<int> devs((size_t)n_scenes);
    for (int r = 0; r < n_scenes; ++r) {
        sc[(size_t)r] = (Scene*)scenes[r];
        if (!sc[(size_t)r]) return fail(PRT_ERR_ARG, "scene handle " + std::to_string(r) + " is NULL");
        devs[(size_t)r] = sc[(size_t)r]->device;
        for (int q = 0; q < r; ++q)
            if (devs[(size_t)q] == devs[(size_t)r])
                return fail(PRT_ERR_ARG, "scene handles must live on distinct devices (device " +
                                             std::to_string(devs[(size_t)r]) + " twice)");
    }
    // tile ownership: the 'latin' interleave of device_scene.tile_owner
    const int tiles_x = (W + tile - 1) / std::max(tile, 1), tiles_y = (H + tile - 1) / std::max(tile, 1);
    const int stride = latin_stride(n_scenes);
    std::vector<std::vector<int32_t>> ids((size_t)n_scenes);
    for (int id = 0; id < tiles_x * tiles_y; ++id)
        ids[(size_t)((id % tiles_x + (int64_t)stride * (id / tiles_x)) % n_scenes)].push_back(id);
    for (int r = 0; r < n_scenes; ++r) {
        int rc = check_render_args(sc[(size_t)r], cam, W, H, tile, tile, ids[(size_t)r].data(),
                                   (int)ids[(size_t)r].size(), spp, depth);
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> lock(g_comm_mu);
    const Rccl& R = rccl();
    if (!R.ok) return fail(PRT_ERR_RCCL, R.why);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        std::vector<ncclComm_t> comms((size_t)n_scenes, nullptr);
        RCCL_TRY(R.comm_init_all(comms.data(), n_scenes, devs.data()));
        it = g_comms.emplace(devs, std::move(comms)).first;
    }
    const std::vector<ncclComm_t>& comms = it->second;
    const int64_t slots = (int64_t)tile * tile;
    const int log_t = __builtin_ctz((unsigned)tile);
    // 1. every rank renders its tiles into its render context's sums (async, own stream)
    std::vector<RenderCtx*> cx((size_t)n_scenes, nullptr);
    std::vector<int64_t> off((size_t)n_scenes + 1, 0);
    for (int r = 0; r < n_scenes; ++r) {
        Scene* s = sc[(size_t)r];
        DeviceGuard g(s->device);
        const int nt = (int)ids[(size_t)r].size();
        off[(size_t)r + 1] = off[(size_t)r] + nt * slots;
        cx[(size_t)r] = ctx_for(s, s->stream);
        if (!cx[(size_t)r]) return fail(PRT_ERR_OOM, "render context allocation failed");
        HIP_TRY(cx[(size_t)r]->acc.ensure(std::max<size_t>(16, sizeof(float) * 3 * (size_t)(nt * slots))));
        int rc = enqueue_render(s, cx[(size_t)r], cam, W, H, tile, tile, ids[(size_t)r].data(), nt, spp, depth, seed,
                                flags, (float*)cx[(size_t)r]->acc.p);
        if (rc) return rc;
    }
    // 2. root buffers: gathered sums of every rank (rank-major) and their tile origins
    Scene* root = sc[0];
    {
        DeviceGuard g(root->device);
        root->gather_xy_host.clear();
        for (int r = 0; r < n_scenes; ++r)
            for (int32_t id : ids[(size_t)r])
                root->gather_xy_host.push_back(((uint32_t)((id % tiles_x) * tile) << 16) |
                                               (uint32_t)((id / tiles_x) * tile));
        HIP_TRY(root->gather.ensure(sizeof(float) * 3 * (size_t)off[(size_t)n_scenes]));
        HIP_TRY(root->gather_xy.ensure(sizeof(uint32_t) * root->gather_xy_host.size()));
        HIP_TRY(root->frame.ensure(sizeof(float) * 3 * (size_t)W * (size_t)H));
        HIP_TRY(hipMemcpyAsync(root->gather_xy.p, root->gather_xy_host.data(),
                               sizeof(uint32_t) * root->gather_xy_host.size(), hipMemcpyHostToDevice, root->stream));
    }
    // 3. the only exchange: every rank (the root too, through its self-loop) sends its packed
    //    tile sums to the root in one RCCL group (point-to-point over xGMI; RCCL has no gather)
    RCCL_TRY(R.group_start());
    for (int r = 0; r < n_scenes; ++r) {
        const size_t n = (size_t)(off[(size_t)r + 1] - off[(size_t)r]) * 3;
        if (n == 0) continue;
        Scene* s = sc[(size_t)r];
        ncclResult_t e = R.send(cx[(size_t)r]->acc.p, n, ncclFloat32, 0, comms[(size_t)r], s->stream);
        if (e == ncclSuccess)
            e = R.recv((float*)root->gather.p + 3 * off[(size_t)r], n, ncclFloat32, r, comms[0], root->stream);
        if (e != ncclSuccess) {
            (void)R.group_end();
            return fail(PRT_ERR_RCCL, std::string("ncclSend/ncclRecv: ") + R.error_string(e));
        }
    }
    RCCL_TRY(R.group_end());
    // 4. root: tiles -> [x][y] frame, frame -> host
    {
        DeviceGuard g(root->device);
        HIP_TRY(prt::launch_scatter((const float*)root->gather.p, (const uint32_t*)root->gather_xy.p,
                                    (int)off[(size_t)n_scenes], log_t, 2 * log_t, 0, 0, W, H, (float*)root->frame.p,
                                    root->stream));
        HIP_TRY(hipMemcpyAsync(out_frame, root->frame.p, sizeof(float) * 3 * (size_t)W * (size_t)H,
                               hipMemcpyDeviceToHost, root->stream));
    }
    for (int r = 0; r < n_scenes; ++r) {
        DeviceGuard g(sc[(size_t)r]->device);
        HIP_TRY(hipStreamSynchronize(sc[(size_t)r]->stream));
        if (take_fault_at(cx[(size_t)r]->work) != 0)
            return fail(PRT_ERR_INTERNAL, "traversal watchdog tripped on device " + std::to_string(devs[(size_t)r]));
    }
    return PRT_OK;
}

void prt_comm_release(void) {
    std::lock_guard<std::mutex> lock(g_comm_mu);
    if (g_rccl.ok)
        for (auto& kv : g_comms)
            for (ncclComm_t c : kv.second) (void)g_rccl.comm_destroy(c);
    g_comms.clear();
}

}  // extern "C"
