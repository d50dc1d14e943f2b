"""A flattened scene resident on one GPU (prt_scene_create / prt_render_tiles*)."""
import ctypes

import numpy as np

from . import _native as N


def tile_grid(W, H, tile):
    tx = (W + tile - 1) // tile
    ty = (H + tile - 1) // tile
    return tx, ty


def latin_stride(world):
    """Row shift s of the 'latin' tile assignment: the integer nearest 0.38 * world
    (a golden-ratio-like step) that is coprime with world, so consecutive tile rows are
    shifted by s and, when world divides the tile columns, every rank owns exactly one
    tile in each run of `world` columns of every row."""
    import math
    s = max(1, int(round(0.38 * world)))
    while math.gcd(s, world) != 1:
        s += 1
    return s


def tile_owner(W, H, tile, world, scheme="latin"):
    """Owner rank of every tile id (ty * tiles_x + tx) — SURVEY.md §8e's interleaving.

    'mod'  : id % world.  On a frame whose tile columns are a multiple of world this
             hands each rank whole tile COLUMNS (8 x 8 tiles at world 8), so ranks see
             different parts of the scene and the slowest one sets the step time.
    'latin': (tx + s * ty) % world with s = latin_stride(world): each rank owns tiles
             spread over every row and column of the frame (a Latin square when world
             divides the tile columns), which evens out the per-rank path cost."""
    tx, ty = tile_grid(W, H, tile)
    ids = np.arange(tx * ty, dtype=np.int64)
    if world <= 1:
        return np.zeros(tx * ty, np.int32)
    if scheme == "mod":
        return (ids % world).astype(np.int32)
    if scheme == "latin":
        return ((ids % tx + latin_stride(world) * (ids // tx)) % world).astype(np.int32)
    raise ValueError(f"unknown tile scheme {scheme!r}")


def interleaved_tiles(W, H, tile, rank=0, world=1, scheme="latin"):
    """Tile ids owned by `rank` of `world`, ascending (see tile_owner)."""
    return np.nonzero(tile_owner(W, H, tile, world, scheme) == rank)[0].astype(np.int32)


def max_tiles_per_rank(W, H, tile, world, scheme="latin"):
    return int(np.bincount(tile_owner(W, H, tile, world, scheme), minlength=max(world, 1)).max())


def unpack_tiles(slots, W, H, tw, th, tile_ids, frame=None):
    """(n_tiles*tw*th, 3) slot sums → (W, H, 3) frame indexed [x][y] (main_taichi.py:25)."""
    tx = (W + tw - 1) // tw
    if frame is None:
        frame = np.zeros((W, H, 3), np.float32)
    s = np.asarray(slots).reshape(len(tile_ids), th, tw, 3)
    for k, tid in enumerate(np.asarray(tile_ids)):
        x0 = (int(tid) % tx) * tw
        y0 = (int(tid) // tx) * th
        w = min(tw, W - x0)
        h = min(th, H - y0)
        frame[x0:x0 + w, y0:y0 + h] = s[k, :h, :w].transpose(1, 0, 2)
    return frame


def pack_rays(o, d, tmin, tmax):
    """(n, 8) float32 ray records (o.xyz, t_min, d.xyz, t_max) of the hit / trace entry points."""
    o = np.asarray(o, np.float32).reshape(-1, 3)
    d = np.asarray(d, np.float32).reshape(-1, 3)
    n = o.shape[0]
    if d.shape[0] != n:
        raise ValueError(f"{n} ray origins but {d.shape[0]} directions")
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = o
    rays[:, 3] = np.broadcast_to(np.asarray(tmin, np.float32), (n,))
    rays[:, 4:7] = d
    rays[:, 7] = np.broadcast_to(np.asarray(tmax, np.float32), (n,))
    return rays


class DeviceScene:
    def __init__(self, flat, device=0):
        self.flat = flat
        self.device = device
        h = ctypes.c_void_p()
        L = N.lib()
        sph = flat.sph if flat.sph.shape[0] else None
        N.check(L.prt_scene_create(device, N.ptr(flat.tri_v), N.ptr(flat.tri_n), N.ptr(flat.tri_mat), flat.n_tri,
                                   N.ptr(sph), N.ptr(flat.sph_mat if sph is not None else None),
                                   flat.sph.shape[0], N.ptr(flat.mat), flat.mat.shape[0], N.ptr(flat.light_tri),
                                   N.ptr(flat.light_off), flat.n_light, N.ptr(flat.direct_rgb), ctypes.byref(h)))
        self.h = h
        info = np.zeros(8, np.int64)
        N.check(L.prt_scene_info(self.h, N.ptr(info)))
        (self.device, self.n_tri, self.n_nodes, self.bvh_depth, self.stack, self.device_bytes, self.blocks_per_cu,
         self.cus) = (int(v) for v in info)

    def close(self):
        if getattr(self, "h", None):
            N.lib().prt_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def render_tiles(self, cam, W, H, tw, th, tile_ids, spp, depth, seed=0, flags=0):
        """Host result: (n_tiles*tw*th, 3) per-pixel radiance sums; returns (sums, stats)."""
        cam = np.ascontiguousarray(cam, np.float32)
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        out = np.zeros((tile_ids.shape[0] * tw * th, 3), np.float32)
        stats = np.zeros(4, np.uint64)
        N.check(N.lib().prt_render_tiles(self.h, N.ptr(cam), W, H, tw, th, N.ptr(tile_ids), tile_ids.shape[0], spp,
                                         depth, int(seed), flags, N.ptr(out), N.ptr(stats)))
        return out, stats

    def render_window(self, cam, W, H, x0, y0, w, h, spp, depth, seed=0, flags=0):
        """prt_render: radiance sums of the window [x0, x0+w) x [y0, y0+h) of a W x H frame,
        (w, h, 3) float32 indexed [x - x0][y - y0]; returns (sums, stats)."""
        cam = np.ascontiguousarray(cam, np.float32)
        out = np.zeros((w, h, 3), np.float32)
        stats = np.zeros(4, np.uint64)
        N.check(N.lib().prt_render(self.h, N.ptr(cam), W, H, x0, y0, w, h, spp, depth, int(seed), flags, N.ptr(out),
                                   N.ptr(stats)))
        return out, stats

    def render_tiles_accumulate(self, cam, W, H, tw, th, tile_ids, first_sample, spp, depth, sums, seed=0, flags=0):
        """Progressive rendering: add samples first_sample .. first_sample+spp-1 onto `sums`
        ((n_tiles*tw*th, 3) float32, modified in place, slot order of render_tiles)."""
        cam = np.ascontiguousarray(cam, np.float32)
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        if sums.dtype != np.float32 or not sums.flags.c_contiguous or sums.shape != (tile_ids.shape[0] * tw * th, 3):
            raise ValueError("sums must be a C-contiguous float32 (n_tiles*tw*th, 3) array")
        N.check(N.lib().prt_render_tiles_accumulate(self.h, N.ptr(cam), W, H, tw, th, N.ptr(tile_ids),
                                                    tile_ids.shape[0], int(first_sample), spp, depth, int(seed), flags,
                                                    N.ptr(sums)))
        return sums

    def render_tiles_device(self, cam, W, H, tw, th, tile_ids, spp, depth, d_out_ptr, stream_ptr=None, seed=0,
                            flags=0):
        """Enqueue; result stays in device memory at d_out_ptr (n_slots x 3 f32)."""
        cam = np.ascontiguousarray(cam, np.float32)
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        N.check(N.lib().prt_render_tiles_device(self.h, N.ptr(cam), W, H, tw, th, N.ptr(tile_ids), tile_ids.shape[0],
                                                spp, depth, int(seed), flags, ctypes.c_void_p(d_out_ptr),
                                                ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def render_frames_device(self, cam, W, H, tw, th, tile_ids, spp, depth, n_frames, d_out_ptr, stream_ptr=None,
                             seed=0, frame_stride=0, flags=0, out_pitch=0):
        """prt_render_frames_device: n_frames frames through the same persistent launches; frame f
        (samples f * frame_stride + 0..spp-1) -> d_out_ptr + f * out_pitch floats (0: packed,
        n_slots * 3 floats).  Enqueued."""
        cam = np.ascontiguousarray(cam, np.float32)
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        N.check(N.lib().prt_render_frames_device(self.h, N.ptr(cam), W, H, tw, th, N.ptr(tile_ids),
                                                 tile_ids.shape[0], spp, depth, int(seed), int(n_frames),
                                                 int(frame_stride), flags, ctypes.c_void_p(d_out_ptr), int(out_pitch),
                                                 ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def scatter_tiles(self, d_packed_ptr, tile_ids, tw, th, W, H, d_frame_ptr, stream_ptr=None):
        """prt_scatter_tiles: packed tile sums (device) -> the device frame (W, H, 3) [x][y], enqueued."""
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        N.check(N.lib().prt_scatter_tiles(self.h, ctypes.c_void_p(d_packed_ptr), N.ptr(tile_ids), tile_ids.shape[0],
                                          tw, th, W, H, ctypes.c_void_p(d_frame_ptr),
                                          ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def scatter_frames(self, d_packed_ptr, tile_ids, group_tiles, group_pitch, tw, th, W, H, n_frames, src_frame_pitch,
                       d_frames_ptr, stream_ptr=None):
        """prt_scatter_frames: a rank-major gather buffer of n_frames frames (rank r's block at
        d_packed + r * group_pitch floats, frame f at + f * src_frame_pitch) -> the device frames
        (n_frames, W, H, 3), one launch.  tile_ids: n_groups * group_tiles host ids, -1 = padding."""
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        if tile_ids.shape[0] % group_tiles:
            raise ValueError("tile_ids must hold whole groups of group_tiles ids")
        N.check(N.lib().prt_scatter_frames(self.h, ctypes.c_void_p(d_packed_ptr), N.ptr(tile_ids),
                                           tile_ids.shape[0] // group_tiles, group_tiles, int(group_pitch), tw, th, W,
                                           H, int(n_frames), int(src_frame_pitch), ctypes.c_void_p(d_frames_ptr),
                                           ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def camera_rays(self, cam, W, H, tw, th, tile_ids, first_sample, spp, seed=0):
        """prt_camera_rays: the primary rays camera_kernel hands the trace kernels, (origin (n, 3),
        direction (n, 3), rng state (n,) u32) in [sample][slot] order."""
        cam = np.ascontiguousarray(cam, np.float32)
        tile_ids = np.ascontiguousarray(tile_ids, np.int32)
        n = tile_ids.shape[0] * tw * th * spp
        out = np.zeros((n, 8), np.float32)
        N.check(N.lib().prt_camera_rays(self.h, N.ptr(cam), W, H, tw, th, N.ptr(tile_ids), tile_ids.shape[0],
                                        int(first_sample), int(spp), int(seed), N.ptr(out)))
        return out[:, 0:3].copy(), out[:, 4:7].copy(), out[:, 3].copy().view(np.uint32)

    def closest_hits(self, o, d, tmin, tmax, any_hit=False, quantized=False):
        """World.hit_all on the GPU for arrays of rays: (hit_id, t); id -1 = miss."""
        rays = pack_rays(o, d, tmin, tmax)
        n = rays.shape[0]
        hid = np.zeros(n, np.int32)
        ht = np.zeros(n, np.float32)
        flags = (N.PRT_HITS_ANY if any_hit else 0) | (N.PRT_HITS_QUANTIZED if quantized else 0)
        N.check(N.lib().prt_closest_hits(self.h, N.ptr(rays), n, flags, N.ptr(hid), N.ptr(ht)))
        return hid, ht

    def hit_all(self, o, d, tmin, tmax, seed=0, quantized=False):
        """prt_hit_all: World.hit_all's 8-tuple per ray as (n, 16) float32 rows — hit, t, p.xyz,
        normal.xyz, emit, attenuation.rgb, scattered direction.xyz, pdf (include/prt.h)."""
        rays = pack_rays(o, d, tmin, tmax)
        out = np.zeros((rays.shape[0], 16), np.float32)
        N.check(N.lib().prt_hit_all(self.h, N.ptr(rays), rays.shape[0], int(seed),
                                    N.PRT_HITS_QUANTIZED if quantized else 0, N.ptr(out)))
        return out

    def trace_rays(self, o, d, depth, seed=0, flags=0):
        """prt_trace_rays: PathTracer.trace's radiance for each caller ray, (n, 3) float32."""
        rays = pack_rays(o, d, 0.0, 0.0)
        out = np.zeros((rays.shape[0], 3), np.float32)
        N.check(N.lib().prt_trace_rays(self.h, N.ptr(rays), rays.shape[0], int(depth), int(seed), flags, N.ptr(out)))
        return out

    def kernel_info(self, n_items=None, flags=0):
        """Trace-kernel variant of a launch of n_items work items (default: a large one) with these
        render flags: dict(variant, bvh_arity, lds_scene, quantized, stack)."""
        out = np.zeros(4, np.int32)
        if n_items is None:
            N.check(N.lib().prt_scene_kernel(self.h, N.ptr(out)))
        else:
            N.check(N.lib().prt_launch_kernel(self.h, int(n_items), flags, N.ptr(out)))
        return dict(variant=int(out[0]), bvh_arity=int(out[1]), lds_scene=bool(out[2] & 1),
                    quantized=bool(out[2] & 2), stack=int(out[3]))

    def kernel_timing(self):
        ms = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        N.check(N.lib().prt_kernel_timing(self.h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def check_faults(self):
        """Synchronise the device and raise PrtError if the traversal watchdog tripped in the
        last render of any of this scene's streams (device-output renders are not checked
        otherwise)."""
        N.check(N.lib().prt_check_faults(self.h))

    def last_stats(self):
        s = np.zeros(4, np.uint64)
        N.check(N.lib().prt_last_stats(self.h, N.ptr(s)))
        return s

    def diag_words(self, n=17):
        """prt_diag_words: the diagnostic words of the last PRT_FLAG_STATS call, [16] = most node
        visits of one query."""
        s = np.zeros(n, np.uint64)
        N.check(N.lib().prt_diag_words(self.h, N.ptr(s), n))
        return s

    def diag_stats(self):
        """16 diagnostic words of the last PRT_FLAG_STATS call (see include/prt.h)."""
        s = np.zeros(16, np.uint64)
        N.check(N.lib().prt_diag_stats(self.h, N.ptr(s)))
        return s


def render_multi(scenes, cam, W, H, tile, spp, depth, seed=0, flags=0):
    """prt_render_multi: the full frame's radiance sums (W, H, 3) [x][y] rendered over the
    devices of `scenes` (DeviceScene handles on distinct GPUs of this process, scenes[0] the
    root), gathered to the root with one RCCL send/recv group."""
    cam = np.ascontiguousarray(cam, np.float32)
    hs = (ctypes.c_void_p * len(scenes))(*[s.h for s in scenes])
    out = np.zeros((W, H, 3), np.float32)
    N.check(N.lib().prt_render_multi(hs, len(scenes), N.ptr(cam), W, H, tile, spp, depth, int(seed), flags,
                                     N.ptr(out)))
    return out
