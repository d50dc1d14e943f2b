/*
 * prt.h — C-ABI of libprt, the MI355X-native path-tracing core behind
 * pyrenderer's Scene / Camera / BSDF API and core.tracing.render().
 *
 * The reference exposes no FFI: its hot path is the Taichi kernel closure
 * `render()` (main_taichi.py:80-99) calling PathTracer.trace
 * (core/tracing.py:116-155) over World.hit_all (mathematics/intersection_taichi.py:238-291),
 * with the scene baked into Taichi fields by World.commit()
 * (mathematics/intersection_taichi.py:220-233) and the camera by
 * Camera.convert_to_taichi_camera() (core/camera.py:27-36).  Each entry point
 * below names the reference interface it replaces; the Python host layer
 * (pyrenderer_amd, ctypes) is the only caller.  INTEGRATION.md shows the
 * binding a pyrenderer maintainer would add.
 *
 * Conventions: all pointers are borrowed for the duration of the call (data is
 * copied to the device); outputs are caller-allocated, C-contiguous float32.
 * Every int-returning function returns PRT_OK (0) or a negative PRT_ERR_*; no
 * C++ exception crosses the ABI; prt_last_error() describes the last failure
 * on the calling thread.  A scene handle is bound to one device and is not
 * re-entrant; distinct handles may be driven from distinct host threads.
 */
#ifndef PRT_H_
#define PRT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.
 * ABI 2: prt_trace_rays, prt_hit_all added; trace-kernel variant ids renumbered to 1..8
 * (PRT_FLAG_VARIANT; 7 / 8 are the pooled-shadow kernel; ids above 8 are rejected with
 * PRT_ERR_ARG, and ABI 1's ids 1..8 named other kernels, so a caller built against ABI 1 must
 * check prt_abi_version()); prt_scene_info's info8[4] is the BVH4 LDS traversal stack depth (0:
 * BVH4 too deep for the LDS-stack variants); watchdog flags are cleared once reported
 * (prt_check_faults).
 * ABI 3 (round 5): prt_render_frames_device (round 4) takes an output pitch between frames
 * (out_pitch, floats; 0 = packed), so a rank whose shard is shorter than its gather slot can render
 * straight into a padded per-frame buffer; prt_scatter_frames and prt_camera_rays added; variant
 * ids 9..14 (three experimental schedules of the pooled kernel) added.
 * ABI 4 (this build, round 6): variant ids 9..14 removed again (none became the default; DESIGN.md
 * §9), ids above 8 are rejected with PRT_ERR_ARG as in ABI 2; prt_scatter_frames rejects a
 * group_pitch too short for n_frames frames at src_frame_pitch; prt_camera_rays zero-fills the rows
 * of slots outside the frame; prt_selftest_guards added. */
#define PRT_ABI_VERSION 4

#define PRT_OK 0
#define PRT_ERR_ARG (-1)     /* invalid argument / shape */
#define PRT_ERR_HIP (-2)     /* HIP runtime error (no device, launch failure, ...) */
#define PRT_ERR_OOM (-3)     /* host or device allocation failed */
#define PRT_ERR_RCCL (-4)    /* RCCL communicator / collective failure */
#define PRT_ERR_UNSUP (-5)   /* feature not supported by this build */
#define PRT_ERR_INTERNAL (-6) /* device-side check failed (traversal watchdog); results invalid */

/* render flags */
#define PRT_FLAG_STATS 0x1u  /* count BVH nodes / triangle tests / queries (slower kernel variant) */
#define PRT_FLAG_TIME 0x2u   /* time the trace kernel with HIP events on its stream */
/* ABI 3: rejected with PRT_ERR_UNSUP — camera rays (and, for cameras other than the affine pinhole,
 * their origins) always come from the camera kernel; the trace kernels carry no camera code, whose
 * uniform operands spilled SGPRs in their loops (C2 4.01 -> 3.91 ms per launch without it) */
#define PRT_FLAG_NO_PRIMARY_KERNEL 0x4u
/* estimator variant: direct lighting by the reference's unused MIS function
 * PathTracer.sample_direct_lighting2 (core/tracing.py:57-90, helpers :12-39) in place of
 * sample_direct_lighting — two closest-hit visibility queries per diffuse vertex (light
 * and BRDF strategies, power heuristic, light_area 1.0 as the reference passes it).
 * A different estimator: the image differs from the default one (oracle: or_set_nee_mode).
 * Selects the MIS kernel variants (4, 5); an explicit variant must agree with the flag. */
#define PRT_FLAG_MIS_NEE 0x8u
/* trace-kernel variant in bits 8..15 (0 = automatic; the numbering is the
 * kVar* table of pyrenderer_amd/csrc/prt_kernels.h: 1 LDS-resident scene (>= 7 waves per
 * SIMD), 2 the same without an occupancy target, 3 global scene (quantised nodes, spill
 * stack), 4 / 5 the MIS estimator on an LDS / global scene, 6 the LDS-resident scene built
 * for >= 6 waves per SIMD, 7 / 8 the LDS-resident block-pooled shadow kernel for >= 7 / >= 6
 * waves per SIMD).  Variants of one estimator produce bit-identical images; the selector exists
 * for A/B runs and tests. */
#define PRT_FLAG_VARIANT_SHIFT 8
#define PRT_FLAG_VARIANT(v) (((uint32_t)(v) & 0xFFu) << PRT_FLAG_VARIANT_SHIFT)

/* material row (8 floats): rho.r rho.g rho.b emit sided type ior roughness */
#define PRT_MAT_LAMBERT 0    /* core/bsdf.py:18-42 BSDFLambertian */
#define PRT_MAT_LIGHT 1      /* core/bsdf.py:45-65 BSDFLight (emit=1, sided=1) */
#define PRT_MAT_METAL 2      /* core/bsdf_taichi.py:45-59 */
#define PRT_MAT_DIELECTRIC 3 /* core/bsdf_taichi.py:62-86 */

/* camera record (24 floats) = CameraTaichi state (core/camera_taichi.py:10-39):
 *   [0:16]  iview_c1..iview_c4 (rows of iview.T)
 *   [16:20] sensor_dim = (sensor_width, sensor_height, focus_dist, aperture)
 *   [20:24] reserved, 0 */
#define PRT_CAM_FLOATS 24

int prt_abi_version(void);
const char* prt_last_error(void);
/* number of visible HIP devices (0 when no GPU; returns PRT_OK either way) */
int prt_device_count(int* n);

/* ---------------------------------------------------------------- BVH ----
 * Replaces accelerators/bvh_taichi.py:107-161 (BVH(prims).build(), median
 * split over primitives) with a binned-SAH BVH2 over triangles.  Host only.
 * tri_v: n_tri x 9 (v0 v1 v2).  info[6] = n_nodes, depth, n_leaves, n_tri,
 * bits of the f32 box padding, round(SAH cost * 1000). */
int prt_bvh_build(const float* tri_v, int64_t n_tri, int32_t max_leaf, void** out_bvh);
int prt_bvh_info(void* bvh, int64_t* info6);
/* nodes: n_nodes x 16 f32; tris: n_tri x 12 f32 (BVH order); order: n_tri (BVH slot -> triangle) */
int prt_bvh_export(void* bvh, float* nodes, float* tris, int32_t* order);
void prt_bvh_destroy(void* bvh);

/* -------------------------------------------------------------- scene ----
 * Replaces World.add / World.commit (mathematics/intersection_taichi.py:220-233)
 * plus the Taichi fields of Quad/Cube (mathematics/shapes.py:49-57, 178-186).
 *   tri_v   n_tri x 9 f32   world-space vertices, face order (v0 v1 v2)
 *   tri_n   n_tri x 3 f32   face normal, reference convention (shapes.py:47,176)
 *   tri_mat n_tri i32       material row
 *   sph     n_sph x 4 f32   center.xyz, radius (intersection_taichi.py:15-36); n_sph may be 0
 *   mat     n_mat x 8 f32   material rows (PRT_MAT_*)
 *   light_tri / light_off   triangles of each emitting primitive, grouped per
 *                           light (light_off has n_light+1 prefix offsets):
 *                           World.sample_a_light + Quad.sample_a_point
 *                           (intersection_taichi.py:194-207, shapes.py:62-71)
 *   direct_rgb 3 f32        colour added when a path hits the light (tracing.py:120)
 * Builds the BVH on the host and uploads everything to `device`. */
int prt_scene_create(int device,
                     const float* tri_v, const float* tri_n, const int32_t* tri_mat, int64_t n_tri,
                     const float* sph, const int32_t* sph_mat, int64_t n_sph,
                     const float* mat, int32_t n_mat,
                     const int32_t* light_tri, const int32_t* light_off, int32_t n_light,
                     const float* direct_rgb, void** out_scene);
/* info[8] = device, n_tri, n_nodes, BVH2 depth, BVH4 LDS traversal stack entries (0: the BVH4 is
 * too deep for the LDS-stack variants, only the spill-stack global variant runs), device
 * bytes, blocks/CU of the default variant, CUs */
int prt_scene_info(void* scene, int64_t* info8);
void prt_scene_destroy(void* scene);

/* ------------------------------------------------------------- render ----
 * Replaces the render() kernel of main_taichi.py:80-99 run `spp` times
 * (pixels[x,y] += PathTracer.trace(...), samples[x,y] += 1).
 * Work = the pixels of `tile_ids` (tiles of tw x th in a W x H frame, tile id =
 * ty * ceil(W/tw) + tx) times samples 0..spp-1, path depth `depth`.
 * out_sum: n_tiles*tw*th x 3 f32, the per-pixel SUM of radiance over samples
 * taken in sample order (divide by spp for the mean: pixels/samples); slot
 * order = tile-major, then row (ly), then column (lx); pixels outside the
 * frame are 0.  Random numbers are keyed by (seed, y*W+x, sample), so the
 * result does not depend on the tiling or on how tiles are spread over GPUs.
 * stats (optional, 4 x u64, needs PRT_FLAG_STATS): BVH nodes visited,
 * triangle tests, extension queries, shadow queries. */
int prt_render_tiles(void* scene, const float* cam, int W, int H, int tw, int th,
                     const int32_t* tile_ids, int n_tiles, int spp, int depth, uint64_t seed,
                     uint32_t flags, float* out_sum, uint64_t* stats);
/* One rectangular window of the frame, as SURVEY.md §8(b)'s prt_render: samples
 * 0..spp-1 of the pixels [x0, x0+w) x [y0, y0+h) of a W x H frame (random streams
 * keyed by the global pixel, so any window equals the same crop of a full-frame render),
 * path depth `depth`.  out_sum: w x h x 3 f32, the per-pixel radiance SUM over samples
 * in sample order, indexed [x - x0][y - y0] like the reference's pixels.to_numpy()
 * (main_taichi.py:25, the render() kernel of main_taichi.py:80-99 run spp times).
 * Rendered as the 8 x 8 tiles covering the window.  stats as prt_render_tiles. */
int prt_render(void* scene, const float* cam, int W, int H, int x0, int y0, int w, int h, int spp, int depth,
               uint64_t seed, uint32_t flags, float* out_sum, uint64_t* stats);
/* The whole W x H frame over several GPUs of this process (SURVEY.md §8(b)
 * prt_render_multi, §8(e)): scenes[r] is a scene handle on its own device (all
 * distinct; scenes[0] is the root).  Tiles of tile x tile pixels go to rank
 * (tx + s*ty) mod n_scenes (the 'latin' interleave of device_scene.tile_owner), every
 * rank renders its tiles on its device, and ONE RCCL group of ncclSend (each rank,
 * the root included) / ncclRecv (root) moves the packed tile sums to the root over
 * xGMI, where they are scattered into out_frame (host, W x H x 3 f32 sums, [x][y]).
 * Bit-identical to prt_render / prt_render_tiles of the same frame for any n_scenes.
 * The communicator (ncclCommInitAll over the scenes' devices) is created on first use
 * and cached per device list; prt_comm_release() destroys the cached ones.  librccl
 * is loaded at first use: PRT_ERR_RCCL when it is missing.  Synchronous. */
int prt_render_multi(void* const* scenes, int n_scenes, const float* cam, int W, int H, int tile, int spp, int depth,
                     uint64_t seed, uint32_t flags, float* out_frame);
void prt_comm_release(void);
/* Root side of a one-process-per-GPU gather (pyrenderer_amd.distributed): the
 * packed tile sums d_packed (device, n_tiles*tw*th x 3 f32, slot order of prt_render_tiles) of the
 * host tile ids `tile_ids` -> the device frame d_frame (W x H x 3 f32, [x][y]; slots outside the
 * frame are dropped, pixels of other tiles untouched), one kernel enqueued on `stream` (NULL = the
 * scene's stream, whose device is used).  A tile id of -1 marks a padding slot (a rank with fewer
 * tiles than the gather buffer's per-rank stride): its pixels are dropped.  The tile origins are
 * uploaded only when the tile set differs from the previous call's.  Replaces a host-side unpack
 * of the gathered buffers. */
int prt_scatter_tiles(void* scene, const float* d_packed, const int32_t* tile_ids, int n_tiles, int tw, int th,
                      int W, int H, float* d_frame, void* stream);
/* ABI 3: the root's scatter of a whole multi-frame gather in ONE launch.  d_packed holds n_groups
 * blocks (one per rank, rank r's at d_packed + r * group_pitch floats), each with n_frames frames of
 * group_tiles tile slots (frame f at + f * src_frame_pitch floats); tile_ids = n_groups * group_tiles
 * host ids (rank-major, -1 = padding).  Frame f goes to d_frames + f * W*H*3 floats ([x][y]).  The
 * launch covers n_groups * group_tiles slots per frame: the per-rank padding of a ragged shard is
 * one tile list, not (world - 1) * n_frames other frames' slots.  ABI 4: with n_groups
 * > 1, group_pitch >= (n_frames - 1) * src_frame_pitch + group_tiles * tw * th * 3, else PRT_ERR_ARG. */
int prt_scatter_frames(void* scene, const float* d_packed, const int32_t* tile_ids, int n_groups, int group_tiles,
                       int64_t group_pitch, int tw, int th, int W, int H, int n_frames, int64_t src_frame_pitch,
                       float* d_frames, void* stream);
/* Progressive rendering: main_taichi.py:108-127 runs render() once per GUI frame
 * (pixels[x,y] += L, samples[x,y] += 1) and displays the running mean.  This call
 * renders samples first_sample .. first_sample+spp-1 of every pixel (the same
 * (seed, pixel, sample) random streams as prt_render_tiles) and adds them, in
 * sample order, onto io_sum (host, n_tiles*tw*th x 3 f32, same slot order):
 * calls covering samples [0, a), [a, b), ... leave io_sum bit-identical to one
 * prt_render_tiles call of b samples.  Synchronous. */
int prt_render_tiles_accumulate(void* scene, const float* cam, int W, int H, int tw, int th,
                                const int32_t* tile_ids, int n_tiles, int first_sample, int spp, int depth,
                                uint64_t seed, uint32_t flags, float* io_sum);
/* Same work, result left in device memory `d_out_sum` (n_slots x 3 f32) and
 * enqueued on `stream` (a hipStream_t; NULL = the scene's own stream) without
 * a host synchronisation. tile_ids is a host array.  The scene keeps one set of
 * work buffers per stream (up to 8), so renders enqueued on distinct streams may
 * execute concurrently on the device (e.g. frame k's drain overlapping frame
 * k+1's start); renders on one stream are ordered as usual.  PRT_FLAG_STATS
 * counters are shared by all streams. */
int prt_render_tiles_device(void* scene, const float* cam, int W, int H, int tw, int th,
                            const int32_t* tile_ids, int n_tiles, int spp, int depth, uint64_t seed,
                            uint32_t flags, float* d_out_sum, void* stream);
/* Several frames through the same persistent launches (the progressive frame loop of
 * main_taichi.py:108-118, or repeated renders of one frame): frame f = samples
 * f * frame_stride + 0 .. spp - 1 of every pixel of the tile set (frame_stride = spp: consecutive
 * progressive frames; 0: n_frames renders of the same samples), its per-pixel sums written to
 * d_out_sums + f * out_pitch floats (device, slot order of prt_render_tiles; out_pitch 0 = packed
 * frames, n_tiles*tw*th*3; otherwise >= that, e.g. the padded per-frame slot of a gather
 * buffer — the floats between a frame's sums and the next frame are not written).  Every frame is
 * bit-identical to the prt_render_tiles_accumulate call of its samples from zero sums; the
 * launches carry all frames' (pixel, sample) items (as many frames per launch as the per-launch
 * buffer budget holds), so a persistent launch ramps up and drains once per launch instead of
 * once per frame.  Enqueued on `stream` like prt_render_tiles_device. */
int prt_render_frames_device(void* scene, const float* cam, int W, int H, int tw, int th,
                             const int32_t* tile_ids, int n_tiles, int spp, int depth, uint64_t seed,
                             int n_frames, int frame_stride, uint32_t flags, float* d_out_sums, int64_t out_pitch,
                             void* stream);
/* trace-kernel time of every render call made with PRT_FLAG_TIME since the
 * previous prt_kernel_timing() (synchronises on their events, then resets):
 * total ms and number of trace launches.  Also reports PRT_ERR_INTERNAL if the
 * traversal watchdog tripped in the last render of any stream (and clears the flags,
 * like prt_check_faults). */
int prt_kernel_timing(void* scene, double* ms_total, int64_t* launches);

/* Self-test of the kernels' exact-reciprocal fast sequence (prt_device.h rcp_fast_seq: v_rcp_f32, one
 * refinement, two corrections) against the IEEE division 1.0f / b for every one of the 2^32 floats
 * on `device`; mismatches8 = mismatches by the class of |b|: 0 zero, 1 denormal, 2 normal < 2^-40,
 * 3 [2^-40, 2^40] (the range the kernels use the sequence in), 4 (2^40, 2^126], 5 > 2^126 finite,
 * 6 infinite, 7 NaN (both results NaN count as equal).  ABI 3, round 5. */
int prt_selftest_rcp(int device, uint64_t* mismatches8);
/* ABI 4: the guards of the kernels' fast sequences, swept over all 2^32 floats b on `device`
 * (counts16, 10 used): 0 rcp_fast_seq mismatches against 1.0f / b that its guard accepts (the result
 * is a normal float) — the kernels rely on this being 0; 1 operands that guard sends to the division;
 * 2 all rcp mismatches; 3 rcp mismatches for normal |b| <= 2^126; 4 sqrt_fast_seq mismatches against
 * sqrtf that its guard accepts (b >= 2^-96) — must be 0; 5 operands sent to sqrtf; 6 all sqrt
 * mismatches; 7 sqrt mismatches in [2^-96, FLT_MAX]; 8 for +0 and normal b < 2^-96; 9 for denormal b
 * (NaN results count as equal). */
int prt_selftest_guards(int device, uint64_t* counts16);
/* Failure detection for renders whose result stays on the device (prt_render_tiles_device,
 * the torch.distributed path): synchronises the device, then reports PRT_ERR_INTERNAL if
 * the traversal watchdog tripped in the last render enqueued on any of this scene's
 * streams.  PRT_OK otherwise.  A flag is cleared once reported — by this call, by
 * prt_kernel_timing, or by the host-output entry points and prt_closest_hits, which check
 * their own launches — so a fault is never reported against a later, clean render. */
int prt_check_faults(void* scene);
/* World.hit_all for a batch of rays (mathematics/intersection_taichi.py:238-291):
 * rays = n x 8 f32 (o.xyz, t_min, d.xyz, t_max); hit_id = original triangle index,
 * n_tri + k for sphere k, -1 for a miss; hit_t = distance (0 on a miss).  Closest hit
 * = minimal (t, id) with the strict t_min < t < t_max test; PRT_HITS_ANY returns
 * some hit in range instead (shadow queries).  PRT_HITS_QUANTIZED traverses the
 * quantised BVH4 of large scenes instead of the f32 one (same results). */
#define PRT_HITS_ANY 0x1u
#define PRT_HITS_QUANTIZED 0x2u
int prt_closest_hits(void* scene, const float* rays, int64_t n, uint32_t flags, int32_t* hit_id, float* hit_t);
/* World.hit_all's full 8-tuple for a batch of rays (mathematics/intersection_taichi.py:238-291,
 * with Quad.hit / Cube.hit's shading at the closest hit, shapes.py:76-110): rays as
 * prt_closest_hits; out = n x 16 f32 per ray:
 *   [0] hit_anything (0/1)  [1] t (closest_so_far: t_max on a miss)  [2:5] p = o + t d
 *   [5:8] normal (flipped toward the ray for two-sided BSDFs, shapes.py:101-102)
 *   [8] emissive (0/1)  [9:12] attenuation = bsdf.evaluate()  [12:15] scattered direction
 *   (cosine-hemisphere draw rotated into the normal frame, bsdf.py:29-34)  [15] pdf = |n.wi|/pi
 * (all zero after [1] on a miss).  The scatter draws 2 numbers from the stream keyed
 * (seed, ray index, 0) — the reference draws them inside hit_all (shapes.py:105) from
 * Taichi's stateful RNG, which cannot be reproduced.  Synchronous. */
int prt_hit_all(void* scene, const float* rays, int64_t n, uint64_t seed, uint32_t flags, float* out16);
/* PathTracer.trace for caller-supplied rays (core/tracing.py:116-155): the radiance of one
 * path per ray, depth `depth`.  rays = n x 8 f32 (o.xyz, unused, d.xyz, unused); out_rgb = n x 3
 * f32.  Ray i draws from the stream keyed (seed, i, 0) — render()'s streams minus the two
 * camera-jitter draws of main_taichi.py:93-94.  flags: PRT_FLAG_MIS_NEE / PRT_FLAG_VARIANT as for
 * the render calls.  Runs the persistent trace kernel of prt_render_tiles.  Synchronous. */
int prt_trace_rays(void* scene, const float* rays, int64_t n, int depth, uint64_t seed, uint32_t flags,
                   float* out_rgb);
/* ABI 3: the primary rays of a render, as camera_kernel generates them for the trace kernels
 * (main_taichi.py:89-95: u = (x + ti.random()) / (W - 1), v likewise, then CameraTaichi.gen_ray
 * core/camera_taichi.py:47-74, the jitter and any lens draws from the stream keyed (seed, pixel,
 * sample)): samples first_sample .. first_sample + spp - 1 of the tile set's pixels, item order
 * [sample][slot] (slot order of prt_render_tiles).  out8 = n x 8 f32: origin.xyz, the RNG state
 * after the camera's draws (u32 bits), direction.xyz, 0.  Parity / inspection entry point (the host
 * gen_ray of PackedCamera is checked against it).  ABI 4: rows of slots whose pixel lies outside
 * the frame (partial edge tiles) are all zeros.  Synchronous. */
int prt_camera_rays(void* scene, const float* cam, int W, int H, int tw, int th, const int32_t* tile_ids,
                    int n_tiles, int first_sample, int spp, uint64_t seed, float* out8);
/* trace-kernel variant chosen for this scene's large launches when flags select none:
 * out4 = {variant, BVH arity (2 or 4), bit 0 scene LDS-resident | bit 1 quantised nodes,
 *         LDS traversal stack entries per lane: the instantiation set, or for the pooled kernel
 *         (7 / 8) the exact BVH4 bound its stack is sized to} */
int prt_scene_kernel(void* scene, int32_t* out4);
/* the same for one trace launch of n_items (pixel, sample) work items with these render flags: an
 * LDS-resident scene whose pool fits seven blocks per CU takes the block-pooled shadow kernel (7) at
 * every launch size (until round 6: the phase-aligned one (1) below eight items per resident lane) */
int prt_launch_kernel(void* scene, int64_t n_items, uint32_t flags, int32_t* out4);
/* counters of the last render call made with PRT_FLAG_STATS (synchronises) */
int prt_last_stats(void* scene, uint64_t* stats4);
/* diagnostic words of the same call (16 x u64): the 4 counters above, then
 * wave-level shader clocks spent in work refill / traversal / shading, wave
 * loop iterations, and active lanes summed over iterations; [11] [12] lane-level
 * inner / leaf traversal trips, [13] deepest traversal stack, [14] samples whose
 * radiance came out NaN or infinite (failure detection; 0 for a sound scene), [15]
 * wave-level triangle-loop trips (max leaf size over the lanes of each leaf trip) */
int prt_diag_stats(void* scene, uint64_t* stats16);
/* the same diagnostic words and any beyond them, n of them (unknown words read 0):
 * [16] most BVH node visits of one query, [23] queries with > 1000 node visits, [24 + 8k ..]
 * the first 16 of them: o.xyz, d.xyz, t_max (f32 bits), query kind << 32 | node visits */
int prt_diag_words(void* scene, uint64_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* PRT_H_ */
